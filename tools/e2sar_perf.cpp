// e2sar_perf -- sender / receiver throughput tool over the reference-shaped C++ API.
//
// The workload and the report follow the reference's bin/e2sar_perf (:123-229 send,
// :279-330 receive; option names :387-423), written against include/e2sar_amd/e2sar.hpp
// to show that a program using e2sar::Segmenter / e2sar::Reassembler the way
// e2sar_perf does runs on the gfx950 path.  Options are parsed by hand (no Boost here).
//
//   e2sar_perf -s -u URI --ip IP -l BYTES -n COUNT -e START -m MTU --rate GBPS --sockets N
//              [--multiport] [--dpv6] [--smooth] [--realmalloc]
//   e2sar_perf -r -u URI --ip IP --port P --threads N --deq N --duration S --timeout MS
//              [--period MS] [-m MTU]
//   e2sar_perf --loopback ...   both sides in one process over 127.0.0.1 (no LB in
//                               between, so the receiver keeps the LB header: withLBHeader)
// Receive slots are sized from -m (a datagram is at most MTU - 28 bytes over IPv4), so a
// 1500-byte MTU does not move 9000-byte slots to the device; a larger datagram is
// truncated and counted in dataErrCnt.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <atomic>
#include <vector>

#include "e2sar_amd/e2sar.hpp"
#include "e2sar_amd/e2sarHeaders.hpp"

using namespace e2sar;
using clk = std::chrono::steady_clock;

namespace {

std::atomic<size_t> sharedReceived{0};   // events received by all dequeue threads

// the reference tool's event payload markers (bin/e2sar_perf.cpp:27-28), so the two tools
// fill events with the same bytes
const std::string kHead = "This is a start of event payload";
const std::string kTail = "...the end";

struct Opts {
    bool send = false, recv = false, loopback = false, quiet = false;
    bool multiport = false, dpv6 = false, smooth = false, realmalloc = false;
    std::string uri, ip = "127.0.0.1";
    size_t length = 1 << 20, num = 10, threads = 1, sockets = 4, deq = 1;
    EventNum_t startEvent = 0;
    uint16_t mtu = 1500, port = 10000, dataId = 4321, lbHdrVersion = 2, periodMs = 1000;
    uint32_t src = 1234;
    float rate = 1.0f;
    int duration = 0, timeoutMs = 500, bufsize = 3 << 20;
    std::string ini;
};

bool parse(int argc, char **argv, Opts &o)
{
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto need = [&](const char *what) -> const char * {
            if (i + 1 >= argc) {
                fprintf(stderr, "option %s needs a value\n", what);
                exit(2);
            }
            return argv[++i];
        };
        if (a == "-s" || a == "--send") o.send = true;
        else if (a == "-r" || a == "--recv") o.recv = true;
        else if (a == "--loopback") o.loopback = true;
        else if (a == "-q" || a == "--quiet") o.quiet = true;
        else if (a == "-u" || a == "--uri") o.uri = need("--uri");
        else if (a == "--ip") o.ip = need("--ip");
        else if (a == "--port") o.port = (uint16_t)atoi(need("--port"));
        else if (a == "-l" || a == "--length") o.length = strtoull(need("--length"), nullptr, 10);
        else if (a == "-n" || a == "--num") o.num = strtoull(need("--num"), nullptr, 10);
        else if (a == "-m" || a == "--mtu") o.mtu = (uint16_t)atoi(need("--mtu"));
        else if (a == "--src") o.src = (uint32_t)strtoul(need("--src"), nullptr, 10);
        else if (a == "--dataid") o.dataId = (uint16_t)atoi(need("--dataid"));
        else if (a == "--lbhdrversion") o.lbHdrVersion = (uint16_t)atoi(need("--lbhdrversion"));
        else if (a == "--threads") o.threads = strtoull(need("--threads"), nullptr, 10);
        else if (a == "--sockets") o.sockets = strtoull(need("--sockets"), nullptr, 10);
        else if (a == "--rate" || a == "--rateGbps") o.rate = (float)atof(need("--rate"));
        else if (a == "-d" || a == "--duration") o.duration = atoi(need("--duration"));
        else if (a == "--timeout") o.timeoutMs = atoi(need("--timeout"));
        else if (a == "-b" || a == "--bufsize") o.bufsize = atoi(need("--bufsize"));
        else if (a == "-i" || a == "--ini") o.ini = need("--ini");
        else if (a == "-e" || a == "--enum") o.startEvent = strtoull(need("--enum"), nullptr, 10);
        else if (a == "--deq") o.deq = strtoull(need("--deq"), nullptr, 10);
        else if (a == "-p" || a == "--period") o.periodMs = (uint16_t)atoi(need("--period"));
        else if (a == "--multiport") o.multiport = true;
        else if (a == "--dpv6") o.dpv6 = true;
        else if (a == "--smooth") o.smooth = true;
        else if (a == "--realmalloc") o.realmalloc = true;
        else {
            fprintf(stderr, "unknown option %s\n", a.c_str());
            return false;
        }
    }
    if ((int)o.send + (int)o.recv + (int)o.loopback != 1) {
        fprintf(stderr, "exactly one of -s, -r, --loopback\n");
        return false;
    }
    // the reference's conflicting_options (bin/e2sar_perf.cpp:440-460)
    if (o.recv && (o.startEvent || o.smooth || o.multiport || o.realmalloc)) {
        fprintf(stderr, "--enum, --smooth, --multiport, --realmalloc are sender options\n");
        return false;
    }
    if (o.send && o.deq != 1) {
        fprintf(stderr, "--deq is a receiver option\n");
        return false;
    }
    if (o.rate < 0 && o.smooth) {
        fprintf(stderr, "--smooth needs a positive --rate\n");
        return false;
    }
    if (o.deq == 0) o.deq = 1;
    if (o.uri.empty())
        o.uri = "ejfat://token@127.0.0.1:18020/lb/1?data=" + o.ip + ":" + std::to_string(o.port);
    return true;
}

// the callback frees the buffer once its last datagram has left (e2sar_perf :117-122)
void freeBuffer(std::any a)
{
    auto p = std::any_cast<uint8_t *>(a);
    if (p) free(p);
}

struct SendResult {
    double seconds = 0;
    size_t events = 0, frames = 0, errors = 0;
};

SendResult sendEvents(Segmenter &s, const Opts &o)
{
    SendResult res;
    const size_t pld = s.getMaxPldLen();
    const size_t expected = o.num * ((o.length + pld - 1) / pld);
    auto open = s.openAndStart();
    if (open.has_error()) {
        fprintf(stderr, "openAndStart: %s\n", open.error().message().c_str());
        exit(1);
    }
    // one event buffer reused for every event unless --realmalloc (bin/e2sar_perf.cpp:
    // 148-170, 664-686); with one buffer nothing is freed by the callback
    uint8_t *one = nullptr;
    if (!o.realmalloc) {
        one = static_cast<uint8_t *>(malloc(o.length));
        memcpy(one, kHead.data(), kHead.size());
        memcpy(one + o.length - kTail.size(), kTail.data(), kTail.size());
    }
    const auto t0 = clk::now();
    size_t evt = 0;
    for (; evt < o.num; evt++) {
        uint8_t *buf = one;
        if (!buf) {
            buf = static_cast<uint8_t *>(malloc(o.length));
            memcpy(buf, kHead.data(), kHead.size());
            memcpy(buf + o.length - kTail.size(), kTail.data(), kTail.size());
        }
        // --enum is the first event number (the reference's loop passes evt itself, :175)
        const EventNum_t en = o.startEvent + evt;
        for (;;) {
            auto r = one ? s.addToSendQueue(buf, o.length, en, 0, 0, nullptr, nullptr)
                         : s.addToSendQueue(buf, o.length, en, 0, 0, &freeBuffer, buf);
            if (!r.has_error()) break;
            if (r.error().code() != E2SARErrorc::MemoryError) {
                fprintf(stderr, "addToSendQueue: %s\n", r.error().message().c_str());
                if (!one) free(buf);
                break;
            }
            std::this_thread::yield();   // queue full, try again (e2sar_perf :176-188)
        }
    }
    for (;;) {
        auto st = s.getSendStats();
        if (st.msgCnt >= expected || st.errCnt > 0) break;
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    res.seconds = std::chrono::duration<double>(clk::now() - t0).count();
    if (one) {
        s.stopThreads();            // every datagram of the shared buffer has left
        free(one);
    }
    auto st = s.getSendStats();
    res.events = evt;
    res.frames = st.msgCnt;
    res.errors = st.errCnt;
    printf("Completed, %zu packets sent, %zu errors\n", (size_t)st.msgCnt, (size_t)st.errCnt);
    printf("Elapsed usecs: %.0f\n", res.seconds * 1e6);
    printf("Estimated effective throughput (Gbps): %.3f\n", st.msgCnt * (double)s.getMTU() * 8.0 / res.seconds / 1e9);
    printf("Estimated goodput (Gbps): %.3f\n", evt * (double)o.length * 8.0 / res.seconds / 1e9);
    return res;
}

struct RecvResult {
    size_t received = 0, mangled = 0, errors = 0, bytes = 0;
    double firstToLast = 0;
};

// One dequeue thread (the reference starts --deq of them, bin/e2sar_perf.cpp:763-769).
RecvResult recvEvents(Reassembler &r, const Opts &o, size_t stopAfter, std::atomic<bool> &stop)
{
    RecvResult res;
    const auto t0 = clk::now();
    clk::time_point first{}, last{};
    while (!stop.load()) {
        uint8_t *buf = nullptr;
        size_t bytes = 0;
        EventNum_t en = 0;
        uint16_t did = 0;
        auto g = r.recvEvent(&buf, &bytes, &en, &did, 1000);
        if (o.duration && clk::now() - t0 > std::chrono::seconds(o.duration)) break;
        if (g.has_error()) {
            res.errors++;
            continue;
        }
        if (g.value() == -1) continue;
        if (!res.received) first = clk::now();
        last = clk::now();
        res.received++;
        res.bytes += bytes;
        if (bytes < kHead.size() + kTail.size() || memcmp(buf, kHead.data(), kHead.size()) ||
            memcmp(buf + bytes - kTail.size(), kTail.data(), kTail.size()))
            res.mangled++;
        delete[] buf;   // ownership passes to the caller (e2sar_perf :299)
        if (stopAfter && sharedReceived.fetch_add(1) + 1 >= stopAfter) stop.store(true);
    }
    res.firstToLast = std::chrono::duration<double>(last - first).count();
    return res;
}

// --deq dequeue threads, results summed
RecvResult recvEventsMT(Reassembler &r, const Opts &o, size_t stopAfter, std::atomic<bool> &stop)
{
    sharedReceived = 0;
    std::vector<RecvResult> rs(o.deq);
    std::vector<std::thread> ts;
    for (size_t i = 0; i < o.deq; i++) ts.emplace_back([&, i] { rs[i] = recvEvents(r, o, stopAfter, stop); });
    // the receive-side reporting thread (bin/e2sar_perf.cpp:306-355), every --period ms
    std::thread rep;
    if (!o.quiet && o.recv)
        rep = std::thread([&] {
            while (!stop.load()) {
                for (int k = 0; k < o.periodMs / 10 && !stop.load(); k++)
                    std::this_thread::sleep_for(std::chrono::milliseconds(10));
                auto st = r.getStats();
                printf("Stats: eventSuccess=%llu enqueueLoss=%llu reassemblyLoss=%llu totalPackets=%zu\n",
                       (unsigned long long)st.eventSuccess, (unsigned long long)st.enqueueLoss,
                       (unsigned long long)st.reassemblyLoss, st.totalPackets);
                fflush(stdout);
            }
        });
    for (auto &t : ts) t.join();
    stop.store(true);
    if (rep.joinable()) rep.join();
    RecvResult all;
    for (const auto &x : rs) {
        all.received += x.received;
        all.mangled += x.mangled;
        all.errors += x.errors;
        all.bytes += x.bytes;
        all.firstToLast = std::max(all.firstToLast, x.firstToLast);
    }
    return all;
}

void printRecv(Reassembler &r, const RecvResult &rr)
{
    auto st = r.getStats();
    printf("Received %zu events (%zu mangled, %zu receive errors)\n", rr.received, rr.mangled, rr.errors);
    printf("Stats: eventSuccess=%llu enqueueLoss=%llu reassemblyLoss=%llu dataErrCnt=%d totalPackets=%zu "
           "totalBytes=%zu badHeaderDiscards=%zu\n",
           (unsigned long long)st.eventSuccess, (unsigned long long)st.enqueueLoss,
           (unsigned long long)st.reassemblyLoss, st.dataErrCnt, st.totalPackets, st.totalBytes,
           st.badHeaderDiscards);
    for (;;) {
        auto l = r.get_LostEvent();
        if (l.has_error()) break;
        printf("Lost event %llu dataId %u fragments %zu\n", (unsigned long long)std::get<0>(l.value()),
               (unsigned)std::get<1>(l.value()), std::get<2>(l.value()));
    }
}

}  // namespace

int main(int argc, char **argv)
{
    Opts o;
    if (!parse(argc, argv, o)) return 2;
    printf("E2SAR Version: %s\n", get_Version().c_str());
    auto uriRes = EjfatURI::getFromString(o.uri, EjfatURI::TokenType::instance);
    if (uriRes.has_error()) {
        fprintf(stderr, "URI: %s\n", uriRes.error().message().c_str());
        return 1;
    }
    const EjfatURI uri = uriRes.value();

    Segmenter::SegmenterFlags sflags;
    Reassembler::ReassemblerFlags rflags;
    if (!o.ini.empty()) {
        if (o.send || o.loopback) {
            auto f = Segmenter::SegmenterFlags::getFromINI(o.ini);
            if (f.has_error()) return fprintf(stderr, "INI: %s\n", f.error().message().c_str()), 1;
            sflags = f.value();
        }
        if (o.recv || o.loopback) {
            auto f = Reassembler::ReassemblerFlags::getFromINI(o.ini);
            if (f.has_error()) return fprintf(stderr, "INI: %s\n", f.error().message().c_str()), 1;
            rflags = f.value();
        }
    } else {
        sflags.useCP = false;
        sflags.mtu = o.mtu;
        sflags.sndSocketBufSize = o.bufsize;
        sflags.numSendSockets = o.sockets;
        sflags.rateGbps = o.rate;
        sflags.lbHdrVersion = (uint8_t)o.lbHdrVersion;
        sflags.multiPort = o.multiport;
        sflags.smooth = o.smooth;
        sflags.dpV6 = o.dpv6;
        rflags.useCP = false;
        rflags.withLBHeader = true;       // back to back: nobody strips the LB header
        rflags.eventTimeout_ms = o.timeoutMs;
        rflags.rcvSocketBufSize = o.bufsize;
        rflags.recvStride = ((size_t)o.mtu - 28 + 15) & ~(size_t)15;
    }

    try {
        if (o.send) {
            Segmenter s(uri, o.dataId, o.src, sflags);
            printf("Event size is %zu bytes, sending %zu events, MTU %u\n", o.length, o.num, s.getMTU());
            sendEvents(s, o);
            s.stopThreads();
            return 0;
        }
        std::atomic<bool> stop{false};
        Reassembler r(uri, o.ip, o.port, o.threads, rflags);
        auto open = r.openAndStart();
        if (open.has_error()) return fprintf(stderr, "openAndStart: %s\n", open.error().message().c_str()), 1;
        printf("Receiving on %s ports %d-%d\n", o.ip.c_str(), r.get_recvPorts().first, r.get_recvPorts().second);
        if (o.recv) {
            auto rr = recvEventsMT(r, o, 0, stop);
            printRecv(r, rr);
            r.stopThreads();
            return 0;
        }
        // loopback: receiver thread + sender here; end-to-end goodput from the first
        // addToSendQueue to the last validated event
        RecvResult rr;
        std::thread rt([&] { rr = recvEventsMT(r, o, o.num, stop); });
        Segmenter s(uri, o.dataId, o.src, sflags);
        printf("Event size is %zu bytes, sending %zu events, MTU %u\n", o.length, o.num, s.getMTU());
        const auto t0 = clk::now();           // after both sides are set up (GPU contexts, buffers)
        sendEvents(s, o);
        // wait for the receiver threads to take every event off the queue (they set `stop`
        // at o.num), bounded by the reassembly timeout plus a margin.  (Waiting on the device
        // counters instead raced the delivery of the last completed events.)
        const auto deadline = clk::now() + std::chrono::milliseconds(2000 + 2 * o.timeoutMs);
        while (clk::now() < deadline && !stop.load())
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        stop.store(true);
        rt.join();
        const double e2e = std::chrono::duration<double>(clk::now() - t0).count();
        printRecv(r, rr);
        printf("End-to-end goodput (Gbps): %.3f (%zu of %zu events intact in %.3f s)\n",
               (rr.received - rr.mangled) * (double)o.length * 8.0 / e2e / 1e9, rr.received - rr.mangled, o.num, e2e);
        s.stopThreads();
        r.stopThreads();
        return (rr.received == o.num && rr.mangled == 0) ? 0 : 3;
    } catch (const E2SARException &e) {
        fprintf(stderr, "E2SARException: %s\n", e.what());
        return 1;
    }
}
