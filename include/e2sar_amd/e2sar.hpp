// e2sar.hpp -- reference-shaped C++ API of the MI355X SAR data path.
//
// The class names, method names, argument meaning and error behaviour follow the
// reference (JeffersonLab/E2SAR v0.3.2):
//   Segmenter    include/e2sarDPSegmenter.hpp:370-553
//   Reassembler  include/e2sarDPReassembler.hpp:383-689
//   errors       include/e2sarError.hpp:23-72 (E2SARErrorc, E2SARErrorInfo, result<T>, E2SARException)
//   EjfatURI     include/e2sarUtil.hpp (only the data/sync address part the data path reads)
// Underneath, every byte of segmentation and reassembly is done by the gfx950 kernels
// behind include/e2sar_hip.h; this layer owns the UDP sockets, the send/recv threads,
// host<->device staging and the reference's queues and counters.
//
// Differences a caller can see (documented in DESIGN.md):
//   - boost::any callback arguments are std::any; boost::tuple results are std::tuple;
//     ip::address arguments are std::string.  Outcome's result<T> is a small local type
//     with the same value()/error()/has_error()/has_value() surface.
//   - No control plane: with useCP the Segmenter runs the reference's Sync thread (a
//     SyncHdr to the URI's sync address every syncPeriodMs, after a warmUpMs warm-up) but
//     talks to no load balancer; registerWorker/deregisterWorker are no-ops that return 0.
//   - SegmenterFlags/ReassemblerFlags gain device fields (gpuDevice, batch sizes, arena).
#pragma once

#include <any>
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <list>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <variant>
#include <vector>

namespace e2sar {

using EventNum_t = uint64_t;

constexpr uint16_t DATAPLANE_PORT = 19522;   // e2sarUtil.hpp:47

enum class E2SARErrorc {
    NoError = 0,
    CaughtException = 1,
    ParseError = 2,
    ParameterError = 3,
    ParameterNotAvailable = 4,
    OutOfRange = 5,
    Undefined = 6,
    NotFound = 7,
    RPCError = 8,
    SocketError = 9,
    MemoryError = 10,
    LogicError = 11,
    SystemError = 12,
    DataError = 13
};

struct E2SARErrorInfo {
    E2SARErrorc ec;
    std::string msg;
    E2SARErrorc code() const { return ec; }
    const std::string &message() const { return msg; }
};

// outcome::result<T, E2SARErrorInfo> surface (e2sarError.hpp:58)
template <class T>
class result {
public:
    result(const T &v) : v_(v) {}
    result(const E2SARErrorInfo &e) : v_(e) {}
    bool has_value() const { return v_.index() == 0; }
    bool has_error() const { return v_.index() == 1; }
    explicit operator bool() const { return has_value(); }
    const T &value() const
    {
        if (!has_value()) throw std::runtime_error("result has no value: " + std::get<1>(v_).msg);
        return std::get<0>(v_);
    }
    const E2SARErrorInfo &error() const
    {
        if (!has_error()) throw std::runtime_error("result has no error");
        return std::get<1>(v_);
    }

private:
    std::variant<T, E2SARErrorInfo> v_;
};

// constructors throw this (e2sarError.hpp:61-72)
class E2SARException : public std::runtime_error {
public:
    explicit E2SARException(const std::string &m) : std::runtime_error(m) {}
    operator std::string() const { return what(); }
};

// The data-path part of EjfatURI: "ejfat[s]://[token@]host:port/lb/<id>?sync=ip:port&data=ip[:port]"
class EjfatURI {
public:
    // e2sarUtil.hpp: token kinds; only the data-path fields of the URI are used here
    enum class TokenType { admin = 0, instance = 1, session = 2 };

    explicit EjfatURI(const std::string &uri, TokenType tt = TokenType::admin, bool preferV6 = false);
    // e2sarUtil.hpp getFromString / getFromEnv: parse errors become E2SARErrorc::ParseError
    static result<EjfatURI> getFromString(const std::string &uri, TokenType tt = TokenType::admin,
                                          bool preferV6 = false) noexcept;
    static result<EjfatURI> getFromEnv(const std::string &envVar = "EJFAT_URI", TokenType tt = TokenType::admin,
                                       bool preferV6 = false) noexcept;
    bool has_dataAddrv4() const { return !dataV4.empty(); }
    bool has_dataAddrv6() const { return !dataV6.empty(); }
    bool has_dataAddr() const { return has_dataAddrv4() || has_dataAddrv6(); }
    bool has_syncAddr() const { return !syncAddr.empty(); }
    result<std::pair<std::string, uint16_t>> get_dataAddrv4() const;
    result<std::pair<std::string, uint16_t>> get_dataAddrv6() const;
    result<std::pair<std::string, uint16_t>> get_syncAddr() const;
    const std::string &get_lbId() const { return lbId; }

private:
    std::string dataV4, dataV6, syncAddr, lbId;
    uint16_t dataV4Port = DATAPLANE_PORT, dataV6Port = DATAPLANE_PORT, syncPort = 0;
};

// get_PortRange (e2sarCP.hpp:772-798)
int get_PortRange(int source_count) noexcept;

// e2sar.hpp get_Version
const std::string get_Version();

// e2sarNetUtil.hpp: the one helper the data-path tools use
namespace NetUtil {
result<std::string> getHostName() noexcept;
// The interface the kernel routes `ip` through and its MTU (e2sarNetUtil.hpp:52,
// e2sarNetUtil.cpp:77): a connected UDP socket selects the route, its local address names
// the interface (getifaddrs), SIOCGIFMTU reads the MTU.  Replaces the reference's
// RTM_GETROUTE netlink query with the same answer for routed destinations.
result<std::tuple<std::string, uint16_t>> getInterfaceAndMTU(const std::string &ip) noexcept;
}

// Flag structs are declared at namespace scope so their default member initialisers
// can serve as default arguments; Segmenter::SegmenterFlags and
// Reassembler::ReassemblerFlags name them as in the reference.
// e2sarDPSegmenter.hpp:370-396 defaults, plus the device fields at the end
struct SegmenterFlagsT {
    bool dpV6{false};
    bool connectedSocket{true};
    bool useCP{true};
    uint16_t warmUpMs{1000};
    uint16_t syncPeriodMs{1000};
    uint16_t syncPeriods{2};
    uint16_t mtu{1500};
    size_t numSendSockets{4};
    int sndSocketBufSize{1024 * 1024 * 3};
    float rateGbps{-1.0};
    bool smooth{false};
    bool multiPort{false};
    bool ticksAsREEventNum{false};
    uint8_t lbHdrVersion{2};
    // device path
    int gpuDevice{0};
    size_t maxBatchEvents{64};            // events segmented per kernel launch (queue path)
    size_t maxBatchBytes{size_t(64) << 20};
    static result<SegmenterFlagsT> getFromINI(const std::string &iniFile) noexcept;
};

// e2sarDPReassembler.hpp:426-450 defaults, plus the device fields at the end
struct ReassemblerFlagsT {
    bool useCP{true};
    bool useHostAddress{false};
    uint16_t period_ms{100};
    bool validateCert{true};
    float Ki{0.}, Kp{0.}, Kd{0.}, setPoint{0.};
    uint32_t epoch_ms{1000};
    int portRange{-1};
    bool withLBHeader{false};
    int eventTimeout_ms{500};
    int rcvSocketBufSize{1024 * 1024 * 3};
    float weight{1.0}, min_factor{0.5}, max_factor{2.0};
    bool reportStats{false};
    // device path
    int gpuDevice{0};
    size_t recvBatch{1024};               // datagrams per reassembly launch
    size_t recvStride{9008};              // bytes per received datagram slot (>= max datagram, x16)
    size_t arenaBytes{size_t(1) << 30};   // device event arena (x2 for compaction)
    uint32_t tableSlots{4096};
    int batchTimeout_us{200};             // flush a partial batch after this long
    // the reference's arrival-order rules on the device (E2SAR_HIP_REAS_REFERENCE_ORDER):
    // offset 0 always starts a new item, completion tested per fragment (cpp:361-427)
    bool referenceOrder{false};
    static result<ReassemblerFlagsT> getFromINI(const std::string &iniFile) noexcept;
};

// ---------------------------------------------------------------------------------

class Segmenter {
public:
    struct ReportedStats {
        uint64_t msgCnt;
        uint64_t errCnt;
        int lastErrno;
        E2SARErrorc lastE2SARError;
    };

    using SegmenterFlags = SegmenterFlagsT;

    Segmenter(const EjfatURI &uri, uint16_t dataId, uint32_t eventSrcId, std::vector<int> cpuCoreList,
              const SegmenterFlags &sflags = SegmenterFlags());
    Segmenter(const EjfatURI &uri, uint16_t dataId, uint32_t eventSrcId,
              const SegmenterFlags &sflags = SegmenterFlags());
    Segmenter(const Segmenter &) = delete;
    Segmenter &operator=(const Segmenter &) = delete;
    ~Segmenter();

    result<int> openAndStart() noexcept;
    result<int> sendEvent(uint8_t *event, size_t bytes, EventNum_t _eventNumber = 0LL, uint16_t _dataId = 0,
                          uint16_t _entropy = 0) noexcept;
    result<int> addToSendQueue(uint8_t *event, size_t bytes, EventNum_t _eventNum = 0LL, uint16_t _dataId = 0,
                               uint16_t entropy = 0, void (*callback)(std::any) = nullptr,
                               std::any cbArg = nullptr) noexcept;
    const ReportedStats getSyncStats() const noexcept;
    const ReportedStats getSendStats() const noexcept;
    const std::string getIntf() const noexcept;
    uint16_t getMTU() const noexcept;
    size_t getMaxPldLen() const noexcept;
    bool isUsingIPv6() const noexcept;
    void stopThreads();

    struct Impl;

private:
    std::unique_ptr<Impl> impl;
};

// ---------------------------------------------------------------------------------

class Reassembler {
public:
    struct ReportedStats {
        EventNum_t enqueueLoss;
        EventNum_t reassemblyLoss;
        EventNum_t eventSuccess;
        int lastErrno;
        int grpcErrCnt;
        int dataErrCnt;
        E2SARErrorc lastE2SARError;
        size_t totalPackets, totalBytes, badHeaderDiscards;
    };

    using ReassemblerFlags = ReassemblerFlagsT;

    Reassembler(const EjfatURI &uri, const std::string &data_ip, uint16_t starting_port,
                std::vector<int> cpuCoreList, const ReassemblerFlags &rflags = ReassemblerFlags());
    Reassembler(const EjfatURI &uri, const std::string &data_ip, uint16_t starting_port,
                size_t numRecvThreads = 1, const ReassemblerFlags &rflags = ReassemblerFlags());
    Reassembler(const EjfatURI &uri, uint16_t starting_port, std::vector<int> cpuCoreList,
                const ReassemblerFlags &rflags = ReassemblerFlags(), bool v6 = false);
    Reassembler(const EjfatURI &uri, uint16_t starting_port, size_t numRecvThreads = 1,
                const ReassemblerFlags &rflags = ReassemblerFlags(), bool v6 = false);
    Reassembler(const Reassembler &) = delete;
    Reassembler &operator=(const Reassembler &) = delete;
    ~Reassembler();

    result<int> registerWorker(const std::string &node_name) noexcept;
    result<int> deregisterWorker() noexcept;
    result<int> openAndStart() noexcept;
    result<int> getEvent(uint8_t **event, size_t *bytes, EventNum_t *eventNum, uint16_t *dataId) noexcept;
    result<int> recvEvent(uint8_t **event, size_t *bytes, EventNum_t *eventNum, uint16_t *dataId,
                          uint64_t wait_ms = 0) noexcept;
    const ReportedStats getStats() const noexcept;
    result<std::tuple<EventNum_t, uint16_t, size_t>> get_LostEvent() noexcept;
    result<std::list<std::pair<uint16_t, size_t>>> get_FDStats() noexcept;
    size_t get_numRecvThreads() const noexcept;
    const std::pair<int, int> get_recvPorts() const noexcept;
    int get_portRange() const noexcept;
    const std::string get_dataIP() const noexcept;
    // device-path diagnostics (no reference counterpart): table / arena occupancy, error
    // flags (bit0 table full, bit1 arena full, bit2 probe timeout) and how many times the
    // table and arena were recycled or compacted
    struct DeviceStats {
        uint64_t tableUsed, arenaUsed, upkeeps;
        int64_t inProgress;
        uint32_t errorFlags;
    };
    const DeviceStats getDeviceStats() const noexcept;
    void stopThreads();

    struct Impl;

private:
    std::unique_ptr<Impl> impl;
};

}  // namespace e2sar
