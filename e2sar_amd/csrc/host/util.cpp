// util.cpp -- EjfatURI (data-path subset), get_PortRange, INI flag loading.
#include <ifaddrs.h>
#include <net/if.h>
#include <sys/ioctl.h>
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>
#include <algorithm>
#include <cctype>
#include <chrono>
#include <cmath>
#include <mutex>
#include <thread>
#include <vector>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <fstream>
#include <map>
#include <sstream>

#include "e2sar_amd/e2sar.hpp"
#include "host_common.hpp"

namespace e2sar {

// "ejfat[s]://[token@]host:port/lb/<id>?sync=ip:port&data=ip[:port]&data=[v6][:port]"
EjfatURI::EjfatURI(const std::string &uri, TokenType, bool)
{
    const auto sch = uri.find("://");
    if (sch == std::string::npos) throw E2SARException("Unable to parse URI: " + uri);
    const std::string scheme = uri.substr(0, sch);
    if (scheme != "ejfat" && scheme != "ejfats") throw E2SARException("Unable to parse URI scheme: " + scheme);
    std::string rest = uri.substr(sch + 3);
    const auto q = rest.find('?');
    const std::string path = rest.substr(0, q);
    const auto lb = path.find("/lb/");
    if (lb != std::string::npos) lbId = path.substr(lb + 4);
    if (q == std::string::npos) return;
    std::stringstream qs(rest.substr(q + 1));
    std::string kv;
    while (std::getline(qs, kv, '&')) {
        const auto eq = kv.find('=');
        if (eq == std::string::npos) continue;
        const std::string k = kv.substr(0, eq), v = kv.substr(eq + 1);
        std::string host;
        uint16_t port = 0;
        bool v6 = false;
        if (!v.empty() && v[0] == '[') {                       // [v6]:port
            const auto rb = v.find(']');
            host = v.substr(1, rb - 1);
            v6 = true;
            if (rb + 1 < v.size() && v[rb + 1] == ':') port = (uint16_t)std::atoi(v.c_str() + rb + 2);
        } else if (std::count(v.begin(), v.end(), ':') > 1) {  // bare v6
            host = v;
            v6 = true;
        } else {
            const auto c = v.find(':');
            host = v.substr(0, c);
            if (c != std::string::npos) port = (uint16_t)std::atoi(v.c_str() + c + 1);
        }
        if (k == "data") {
            if (v6) {
                dataV6 = host;
                dataV6Port = port ? port : DATAPLANE_PORT;
            } else {
                dataV4 = host;
                dataV4Port = port ? port : DATAPLANE_PORT;
            }
        } else if (k == "sync") {
            syncAddr = host;
            syncPort = port;
        }
    }
}

result<std::pair<std::string, uint16_t>> EjfatURI::get_dataAddrv4() const
{
    if (dataV4.empty()) return E2SARErrorInfo{E2SARErrorc::ParameterNotAvailable, "Data address not present"};
    return std::make_pair(dataV4, dataV4Port);
}

result<std::pair<std::string, uint16_t>> EjfatURI::get_dataAddrv6() const
{
    if (dataV6.empty()) return E2SARErrorInfo{E2SARErrorc::ParameterNotAvailable, "Data address not present"};
    return std::make_pair(dataV6, dataV6Port);
}

result<std::pair<std::string, uint16_t>> EjfatURI::get_syncAddr() const
{
    if (syncAddr.empty()) return E2SARErrorInfo{E2SARErrorc::ParameterNotAvailable, "Sync address not present"};
    return std::make_pair(syncAddr, syncPort);
}

// e2sarCP.hpp:772-798
int get_PortRange(int source_count) noexcept
{
    if (source_count < 2) return 0;
    if (source_count > 16384) return 14;
    int maxCount = 2, iteration = 1;
    while (source_count > maxCount) {
        iteration++;
        maxCount <<= 1;
    }
    return iteration;
}

namespace detail {

float clock_entropy_bits()
{
    static std::once_flag once;
    static float bits = 0.0f;
    std::call_once(once, [] {
        constexpr int kTests = 1000;
        std::vector<int> bins(256, 0);
        for (int i = 0; i < kTests; i++) {
            const auto now = std::chrono::system_clock::now();
            bins[std::chrono::duration_cast<std::chrono::microseconds>(now.time_since_epoch()).count() & 0xff]++;
            std::this_thread::sleep_until(now + std::chrono::milliseconds(1));
        }
        double e = 0.0;
        for (int b : bins)
            if (b) {
                const double p = (double)b / kTests;
                e -= p * std::log(p);
            }
        bits = (float)(e / std::log(2.0));
    });
    return bits;
}

static std::string trim(const std::string &s)
{
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) a++;
    while (b > a && std::isspace((unsigned char)s[b - 1])) b--;
    return s.substr(a, b - a);
}

bool read_ini(const std::string &path, std::map<std::string, std::string> &out, std::string &err)
{
    std::ifstream f(path);
    if (!f) {
        err = "Unable to open INI file " + path;
        return false;
    }
    std::string line, section;
    while (std::getline(f, line)) {
        line = trim(line);
        if (line.empty() || line[0] == ';' || line[0] == '#') continue;
        if (line.front() == '[' && line.back() == ']') {
            section = trim(line.substr(1, line.size() - 2));
            continue;
        }
        const auto eq = line.find('=');
        if (eq == std::string::npos) {
            err = "Unable to parse INI line: " + line;
            return false;
        }
        out[section + "." + trim(line.substr(0, eq))] = trim(line.substr(eq + 1));
    }
    return true;
}

bool ini_bool(const std::map<std::string, std::string> &m, const std::string &k, bool def)
{
    auto it = m.find(k);
    if (it == m.end()) return def;
    return it->second == "true" || it->second == "1" || it->second == "yes";
}

double ini_num(const std::map<std::string, std::string> &m, const std::string &k, double def)
{
    auto it = m.find(k);
    if (it == m.end()) return def;
    return std::atof(it->second.c_str());
}

}  // namespace detail

// e2sarDPSegmenter.cpp:950-996 (warmUpMS read as a number here; the reference reads it as bool)
result<SegmenterFlagsT> SegmenterFlagsT::getFromINI(const std::string &iniFile) noexcept
{
    std::map<std::string, std::string> m;
    std::string err;
    if (!detail::read_ini(iniFile, m, err)) return E2SARErrorInfo{E2SARErrorc::ParameterNotAvailable, err};
    SegmenterFlagsT f;
    f.useCP = detail::ini_bool(m, "general.useCP", f.useCP);
    f.warmUpMs = (uint16_t)detail::ini_num(m, "control-plane.warmUpMS", f.warmUpMs);
    f.syncPeriods = (uint16_t)detail::ini_num(m, "control-plane.syncPeriods", f.syncPeriods);
    f.syncPeriodMs = (uint16_t)detail::ini_num(m, "control-plane.syncPeriodMS", f.syncPeriodMs);
    f.dpV6 = detail::ini_bool(m, "data-plane.dpV6", f.dpV6);
    f.connectedSocket = detail::ini_bool(m, "data-plane.connectedSocket", f.connectedSocket);
    f.ticksAsREEventNum = detail::ini_bool(m, "data-plane.ticksAsREEventNum", f.ticksAsREEventNum);
    f.mtu = (uint16_t)detail::ini_num(m, "data-plane.mtu", f.mtu);
    f.numSendSockets = (size_t)detail::ini_num(m, "data-plane.numSendSockets", (double)f.numSendSockets);
    f.sndSocketBufSize = (int)detail::ini_num(m, "data-plane.sndSocketBufSize", f.sndSocketBufSize);
    f.rateGbps = (float)detail::ini_num(m, "data-plane.rateGbps", f.rateGbps);
    f.smooth = detail::ini_bool(m, "data-plane.smooth", f.smooth);
    f.multiPort = detail::ini_bool(m, "data-plane.multiPort", f.multiPort);
    f.lbHdrVersion = (uint8_t)detail::ini_num(m, "data-plane.lbHdrVersion", f.lbHdrVersion);
    f.gpuDevice = (int)detail::ini_num(m, "device.gpuDevice", f.gpuDevice);
    f.maxBatchEvents = (size_t)detail::ini_num(m, "device.maxBatchEvents", (double)f.maxBatchEvents);
    return f;
}

// e2sarDPReassembler.cpp:678-719 (the PID weights go to their own fields here; the
// reference assigns pid.weight/min_factor/max_factor to Kd)
result<ReassemblerFlagsT> ReassemblerFlagsT::getFromINI(const std::string &iniFile) noexcept
{
    std::map<std::string, std::string> m;
    std::string err;
    if (!detail::read_ini(iniFile, m, err)) return E2SARErrorInfo{E2SARErrorc::ParameterNotAvailable, err};
    ReassemblerFlagsT f;
    f.useCP = detail::ini_bool(m, "general.useCP", f.useCP);
    f.useHostAddress = detail::ini_bool(m, "control-plane.useHostAddress", f.useHostAddress);
    f.validateCert = detail::ini_bool(m, "control-plane.validateCert", f.validateCert);
    f.reportStats = detail::ini_bool(m, "control-plane.reportStats", f.reportStats);
    f.portRange = (int)detail::ini_num(m, "data-plane.portRange", f.portRange);
    f.withLBHeader = detail::ini_bool(m, "data-plane.withLBHeader", f.withLBHeader);
    f.eventTimeout_ms = (int)detail::ini_num(m, "data-plane.eventTimeoutMS", f.eventTimeout_ms);
    f.rcvSocketBufSize = (int)detail::ini_num(m, "data-plane.rcvSocketBufSize", f.rcvSocketBufSize);
    f.epoch_ms = (uint32_t)detail::ini_num(m, "data-plane.epochMS", f.epoch_ms);
    f.period_ms = (uint16_t)detail::ini_num(m, "data-plane.periodMS", f.period_ms);
    f.setPoint = (float)detail::ini_num(m, "pid.setPoint", f.setPoint);
    f.Ki = (float)detail::ini_num(m, "pid.Ki", f.Ki);
    f.Kp = (float)detail::ini_num(m, "pid.Kp", f.Kp);
    f.Kd = (float)detail::ini_num(m, "pid.Kd", f.Kd);
    f.weight = (float)detail::ini_num(m, "pid.weight", f.weight);
    f.min_factor = (float)detail::ini_num(m, "pid.min_factor", f.min_factor);
    f.max_factor = (float)detail::ini_num(m, "pid.max_factor", f.max_factor);
    f.gpuDevice = (int)detail::ini_num(m, "device.gpuDevice", f.gpuDevice);
    f.recvBatch = (size_t)detail::ini_num(m, "device.recvBatch", (double)f.recvBatch);
    f.arenaBytes = (size_t)detail::ini_num(m, "device.arenaBytes", (double)f.arenaBytes);
    f.recvStride = (size_t)detail::ini_num(m, "device.recvStride", (double)f.recvStride);
    f.tableSlots = (uint32_t)detail::ini_num(m, "device.tableSlots", (double)f.tableSlots);
    f.referenceOrder = detail::ini_num(m, "device.referenceOrder", f.referenceOrder ? 1.0 : 0.0) != 0.0;
    return f;
}

}  // namespace e2sar

namespace e2sar {

result<EjfatURI> EjfatURI::getFromString(const std::string &uri, TokenType tt, bool preferV6) noexcept
{
    try {
        return EjfatURI(uri, tt, preferV6);
    } catch (const std::exception &e) {
        return E2SARErrorInfo{E2SARErrorc::ParseError, e.what()};
    }
}

result<EjfatURI> EjfatURI::getFromEnv(const std::string &envVar, TokenType tt, bool preferV6) noexcept
{
    const char *v = std::getenv(envVar.c_str());
    if (!v) return E2SARErrorInfo{E2SARErrorc::Undefined, "environment variable " + envVar + " not defined"};
    return getFromString(v, tt, preferV6);
}

const std::string get_Version() { return "0.3.2-mi355x"; }

namespace NetUtil {
result<std::string> getHostName() noexcept
{
    char buf[256];
    if (gethostname(buf, sizeof(buf)) != 0) return E2SARErrorInfo{E2SARErrorc::SystemError, strerror(errno)};
    buf[sizeof(buf) - 1] = 0;
    return std::string(buf);
}
result<std::tuple<std::string, uint16_t>> getInterfaceAndMTU(const std::string &ip) noexcept
{
    const bool v6 = ip.find(':') != std::string::npos;
    sockaddr_storage ss{};
    socklen_t sl;
    if (v6) {
        auto *a = reinterpret_cast<sockaddr_in6 *>(&ss);
        a->sin6_family = AF_INET6;
        a->sin6_port = htons(9);
        if (inet_pton(AF_INET6, ip.c_str(), &a->sin6_addr) != 1) return E2SARErrorInfo{E2SARErrorc::ParameterError, "bad IPv6 address " + ip};
        sl = sizeof(sockaddr_in6);
    } else {
        auto *a = reinterpret_cast<sockaddr_in *>(&ss);
        a->sin_family = AF_INET;
        a->sin_port = htons(9);
        if (inet_pton(AF_INET, ip.c_str(), &a->sin_addr) != 1) return E2SARErrorInfo{E2SARErrorc::ParameterError, "bad IPv4 address " + ip};
        sl = sizeof(sockaddr_in);
    }
    const int fd = socket(v6 ? AF_INET6 : AF_INET, SOCK_DGRAM, 0);
    if (fd < 0) return E2SARErrorInfo{E2SARErrorc::SocketError, strerror(errno)};
    // connect() on a UDP socket sends nothing; it makes the kernel pick the route
    sockaddr_storage local{};
    socklen_t ll = sizeof(local);
    if (connect(fd, reinterpret_cast<sockaddr *>(&ss), sl) != 0 ||
        getsockname(fd, reinterpret_cast<sockaddr *>(&local), &ll) != 0) {
        const std::string err = strerror(errno);
        close(fd);
        return E2SARErrorInfo{E2SARErrorc::SocketError, "no route to " + ip + ": " + err};
    }
    ifaddrs *ifa = nullptr;
    if (getifaddrs(&ifa) != 0) {
        close(fd);
        return E2SARErrorInfo{E2SARErrorc::SocketError, strerror(errno)};
    }
    std::string name;
    for (ifaddrs *i = ifa; i && name.empty(); i = i->ifa_next) {
        if (!i->ifa_addr || i->ifa_addr->sa_family != local.ss_family) continue;
        if (v6) {
            if (!memcmp(&reinterpret_cast<sockaddr_in6 *>(i->ifa_addr)->sin6_addr,
                        &reinterpret_cast<sockaddr_in6 *>(&local)->sin6_addr, sizeof(in6_addr)))
                name = i->ifa_name;
        } else if (reinterpret_cast<sockaddr_in *>(i->ifa_addr)->sin_addr.s_addr ==
                   reinterpret_cast<sockaddr_in *>(&local)->sin_addr.s_addr) {
            name = i->ifa_name;
        }
    }
    freeifaddrs(ifa);
    if (name.empty()) {
        close(fd);
        return E2SARErrorInfo{E2SARErrorc::NotFound, "no interface holds the local address routed to " + ip};
    }
    ifreq ifr{};
    strncpy(ifr.ifr_name, name.c_str(), IFNAMSIZ - 1);
    const int rc = ioctl(fd, SIOCGIFMTU, &ifr);
    close(fd);
    if (rc != 0) return E2SARErrorInfo{E2SARErrorc::SocketError, std::string("SIOCGIFMTU: ") + strerror(errno)};
    // the MTU travels as u_int16_t, as in the reference (e2sarNetUtil.cpp:147-149 narrows
    // getMTU's size_t): loopback's 65536 reads as 0 there ("lo doesn't" report one,
    // e2sarDPSegmenter.cpp:86-88), and so it does here
    return std::make_tuple(name, (uint16_t)ifr.ifr_mtu);
}

}  // namespace NetUtil

}  // namespace e2sar
