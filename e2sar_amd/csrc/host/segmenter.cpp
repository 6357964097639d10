// segmenter.cpp -- e2sar::Segmenter over the gfx950 segmentation kernel.
//
// The reference segments one event at a time on a CPU thread pool and hands every
// datagram to the kernel with its own sendmsg (e2sarDPSegmenter.cpp:375-468, 660-871).
// Here the send thread drains the event queue in batches: the batch's events are copied
// to HBM once, seg_kernel writes every datagram of the batch in one launch, the datagram
// batch comes back to pinned memory in one copy and leaves through sendmmsg, one call
// per event on a round-robin socket (the reference's sendmmsg optimisation, :772-857).
// sendEvent() is the synchronous single-event form (cpp:901-917).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <random>
#include <thread>

#include "e2sar_amd/e2sarHeaders.hpp"
#include "host_common.hpp"

namespace e2sar {

using detail::hip_error;

constexpr float kMinClockEntropy = 6.0f;   // MIN_CLOCK_ENTROPY (e2sarDPSegmenter.hpp:293)

struct Segmenter::Impl {
    EjfatURI uri;
    uint16_t dataId;
    uint32_t eventSrcId;
    SegmenterFlags flags;
    std::vector<int> cores;
    bool useV6 = false;
    uint16_t mtu = 1500;
    std::string iface;               // outgoing interface of the data address (getIntf)
    size_t maxPld = 0;
    uint32_t stride = 0;

    // device + staging
    e2sar_hip_ctx *ctx = nullptr;
    void *stream = nullptr;
    uint8_t *dEvents = nullptr;
    size_t dEventsCap = 0;
    e2sar_hip_seg_event *dDesc = nullptr;
    size_t dDescCap = 0;
    uint8_t *dPkts = nullptr;
    uint32_t *dLens = nullptr;
    uint8_t *hPkts = nullptr;
    uint32_t *hLens = nullptr;
    size_t pktCap = 0;
    std::vector<e2sar_hip_seg_event> hDesc;
    std::mutex devMu;

    // sockets
    std::vector<int> fds;
    std::vector<sockaddr_storage> dsts;
    socklen_t dstLen = 0;
    size_t rr = 0;

    // stats (e2sarDPSegmenter.hpp:149-161)
    std::atomic<uint64_t> msgCnt{0}, errCnt{0};
    std::atomic<int> lastErrno{0};
    std::atomic<E2SARErrorc> lastErr{E2SARErrorc::NoError};
    std::atomic<EventNum_t> userEventNum{0};

    // Sync thread (useCP): a SyncHdr to the URI's sync address every syncPeriodMs
    // (e2sarDPSegmenter.cpp:242-373, fillSyncHdr hpp:583-591)
    int syncFd = -1;
    sockaddr_storage syncDst{};
    socklen_t syncDstLen = 0;
    std::thread syncThread;
    std::mutex syncMu;
    std::condition_variable syncCv;
    bool syncStop = false;
    std::atomic<uint64_t> syncMsgCnt{0}, syncErrCnt{0};
    std::atomic<int> syncLastErrno{0};

    // send queue (lock-free queue of 2047 items in the reference, hpp:81,101)
    struct Item {
        uint8_t *event;
        size_t bytes;
        EventNum_t eventNum;
        uint16_t dataId;
        uint16_t entropy;
        void (*cb)(std::any);
        std::any cbArg;
    };
    static constexpr size_t kQueueCap = 2047;
    std::mutex qMu;
    std::condition_variable qCv, qEmptyCv;
    std::deque<Item> q;
    size_t inFlight = 0;
    std::thread sendThread;
    std::atomic<bool> stop{false};
    bool started = false;
    std::mt19937 rng{std::random_device{}()};
    bool addEntropy = false;                              // clock LSBs need help (cpp:50)
    std::chrono::steady_clock::time_point paceNext{};   // rate pacing: earliest start of the next event

    Impl(const EjfatURI &u, uint16_t did, uint32_t esid, std::vector<int> c, const SegmenterFlags &f)
        : uri(u), dataId(did), eventSrcId(esid), flags(f), cores(std::move(c))
    {
    }
    ~Impl();

    void sanity();
    result<int> ensure(size_t eventBytes, size_t nEvents, size_t nPackets);
    result<int> sendBatch(std::vector<Item> &items);
    void threadBody();
    result<int> syncOpen();
    void syncSend();
    void syncBody();
    void syncHalt();
};

Segmenter::Impl::~Impl()
{
    syncHalt();
    for (int fd : fds) close(fd);
    if (ctx) {
        e2sar_hip_stream_sync(ctx, stream);
        if (dEvents) e2sar_hip_device_free(ctx, dEvents);
        if (dDesc) e2sar_hip_device_free(ctx, dDesc);
        if (dPkts) e2sar_hip_device_free(ctx, dPkts);
        if (dLens) e2sar_hip_device_free(ctx, dLens);
        if (hPkts) e2sar_hip_host_free(hPkts);
        if (hLens) e2sar_hip_host_free(hLens);
        e2sar_hip_ctx_destroy(ctx);
    }
    if (stream) e2sar_hip_stream_destroy(stream);
}

namespace detail {
// e2sarDPSegmenter.cpp:56-110: mtu 0 takes the outgoing interface's MTU as reported; an
// override must not exceed it (an interface that reports 0 accepts any override)
uint32_t resolve_mtu(uint16_t flagsMtu, uint32_t ifMtu, const std::string &iface)
{
    if (flagsMtu == 0) {
        if (ifMtu == 0) throw E2SARException("Outgoing interface MTU is reported as 0, please use manual override of MTU size");
        return ifMtu;
    }
    if (ifMtu > 0 && flagsMtu > ifMtu)
        throw E2SARException("Segmenter flags MTU override value exceeds outgoing interface MTU of " + iface);
    return flagsMtu;
}

// e2sarDPSegmenter.hpp:307-308, applied to the resolved MTU: an auto-detected 9216 (jumbo
// Ethernet) or 65520 (IPoIB) is refused like an override above 9000, so the datagram slots
// never outgrow the 9000-byte layout the data plane is sized for
void check_mtu_limit(uint32_t mtu)
{
    if (mtu > 9000) throw E2SARException("MTU set too long, limit 9000");
}

// addToSendQueue's numbering (cpp:925-937): an explicit number resets the counter, and the
// number is taken before the push can fail (cpp:939-946), so a refused default-numbered
// event leaves a gap.  Returns the number taken; *accepted says whether a queue holding
// `depth` items of `cap` takes the event.
EventNum_t take_send_number(std::atomic<EventNum_t> &userEventNum, EventNum_t eventNum, size_t depth, size_t cap,
                            bool *accepted)
{
    if (eventNum != 0) userEventNum.exchange(eventNum);
    const EventNum_t num = userEventNum++;
    *accepted = depth < cap;
    return num;
}
}  // namespace detail

// e2sarDPSegmenter.hpp:298-317 + ctor checks at cpp:52-53
void Segmenter::Impl::sanity()
{
    if (flags.lbHdrVersion < 2 || flags.lbHdrVersion > 3)
        throw E2SARException("Only allowed LB header version numbers are 2 or 3");
    if (flags.numSendSockets > 128) throw E2SARException("Too many sending sockets threads requested, limit 128");
    if (flags.numSendSockets == 0) throw E2SARException("At least one sending socket is required");
    if (flags.syncPeriodMs > 10000) throw E2SARException("Sync period too long, limit 10s");
    detail::check_mtu_limit(mtu);          // the resolved MTU, as the reference checks it (hpp:307)
    if (flags.useCP && !uri.has_syncAddr()) throw E2SARException("Sync address not present in the URI");
    if (!uri.has_dataAddr()) throw E2SARException("Data address is not present in the URI");
    if (mtu <= e2sar_hip_total_hdr_len(useV6 ? 1 : 0))
        throw E2SARException("Insufficient MTU length to accommodate headers");
}

static void init_impl(Segmenter::Impl &m)
{
    m.useV6 = m.flags.dpV6 && m.uri.has_dataAddrv6();
    if (!m.uri.has_dataAddrv4() && m.uri.has_dataAddrv6()) m.useV6 = true;
    // outgoing interface and its MTU for the URI's data address (e2sarDPSegmenter.cpp:56-110),
    // with the reference's rules: a failed lookup throws whatever the override; mtu 0 takes
    // the interface's MTU as reported (loopback's 65536 reads as 0 through the reference's
    // u_int16_t, e2sarNetUtil.cpp:147-149, and is refused; a jumbo 9216 fails the 9000-byte
    // check in sanity(), hpp:307-308); an override must not exceed the interface's MTU.
    auto addr = m.useV6 ? m.uri.get_dataAddrv6() : m.uri.get_dataAddrv4();
    if (addr.has_error()) throw E2SARException("Data address is not present in the URI");
    auto intf = NetUtil::getInterfaceAndMTU(addr.value().first);
    if (!intf.has_value())
        throw E2SARException("Unable to determine outgoing interface for LB destination address " +
                             addr.value().first + ": " + intf.error().message());
    m.iface = std::get<0>(intf.value());
    m.mtu = detail::resolve_mtu(m.flags.mtu, std::get<1>(intf.value()), m.iface);
    m.sanity();
    m.maxPld = e2sar_hip_max_pld_len(m.mtu, m.useV6 ? 1 : 0);     // cpp:113
    m.addEntropy = !(detail::clock_entropy_bits() > kMinClockEntropy);   // cpp:50
    m.stride = e2sar_hip_packet_stride(m.maxPld);
    int rc = e2sar_hip_stream_create(m.flags.gpuDevice, &m.stream);
    if (rc == 0) rc = e2sar_hip_ctx_create(m.flags.gpuDevice, m.stream, &m.ctx);
    if (rc) throw E2SARException(std::string("Unable to open GPU ") + std::to_string(m.flags.gpuDevice) + ": " +
                                 e2sar_hip_last_error());
}

Segmenter::Segmenter(const EjfatURI &uri, uint16_t dataId, uint32_t eventSrcId, std::vector<int> cpuCoreList,
                     const SegmenterFlags &sflags)
    : impl(new Impl(uri, dataId, eventSrcId, std::move(cpuCoreList), sflags))
{
    init_impl(*impl);
}

Segmenter::Segmenter(const EjfatURI &uri, uint16_t dataId, uint32_t eventSrcId, const SegmenterFlags &sflags)
    : impl(new Impl(uri, dataId, eventSrcId, {}, sflags))
{
    init_impl(*impl);
}

Segmenter::~Segmenter() { stopThreads(); }

result<int> Segmenter::Impl::ensure(size_t eventBytes, size_t nEvents, size_t nPackets)
{
    int rc;
    if (eventBytes > dEventsCap) {
        if (dEvents) e2sar_hip_device_free(ctx, dEvents);
        dEventsCap = std::max(eventBytes, dEventsCap * 2);
        if ((rc = e2sar_hip_device_alloc(ctx, dEventsCap, reinterpret_cast<void **>(&dEvents)))) {
            dEventsCap = 0;
            return hip_error(rc, "device event staging");
        }
    }
    if (nEvents > dDescCap) {
        if (dDesc) e2sar_hip_device_free(ctx, dDesc);
        dDescCap = std::max<size_t>(nEvents, 64);
        if ((rc = e2sar_hip_device_alloc(ctx, dDescCap * sizeof(e2sar_hip_seg_event),
                                         reinterpret_cast<void **>(&dDesc)))) {
            dDescCap = 0;
            return hip_error(rc, "device event table");
        }
    }
    if (nPackets > pktCap) {
        if (dPkts) e2sar_hip_device_free(ctx, dPkts);
        if (dLens) e2sar_hip_device_free(ctx, dLens);
        if (hPkts) e2sar_hip_host_free(hPkts);
        if (hLens) e2sar_hip_host_free(hLens);
        dPkts = hPkts = nullptr;
        dLens = hLens = nullptr;
        pktCap = std::max(nPackets, pktCap * 2);
        if ((rc = e2sar_hip_device_alloc(ctx, pktCap * stride, reinterpret_cast<void **>(&dPkts))) ||
            (rc = e2sar_hip_device_alloc(ctx, pktCap * 4, reinterpret_cast<void **>(&dLens))) ||
            (rc = e2sar_hip_host_alloc(pktCap * stride, reinterpret_cast<void **>(&hPkts))) ||
            (rc = e2sar_hip_host_alloc(pktCap * 4, reinterpret_cast<void **>(&hLens)))) {
            pktCap = 0;
            return hip_error(rc, "datagram staging");
        }
    }
    return 0;
}

// Segment + send one batch of events (the _send body for many events at once).
result<int> Segmenter::Impl::sendBatch(std::vector<Item> &items)
{
    std::lock_guard<std::mutex> lk(devMu);
    hDesc.resize(items.size());
    size_t total = 0;
    for (size_t i = 0; i < items.size(); i++) {
        if (items[i].bytes >= (size_t(1) << 32))
            return E2SARErrorInfo{E2SARErrorc::ParameterError, "event larger than 4 GiB (REHdr bufferLength is u32)"};
        total = (total + 15) & ~size_t(15);
        hDesc[i].data = reinterpret_cast<const uint8_t *>(total);   // offset for now
        total += items[i].bytes;
    }
    uint32_t nPk = 0, maxPk = 0;
    for (size_t i = 0; i < items.size(); i++) hDesc[i].bytes = (uint32_t)items[i].bytes;
    int rc = e2sar_hip_seg_plan(hDesc.data(), (uint32_t)items.size(), maxPld, &nPk, &maxPk);
    if (rc) return hip_error(rc, "seg_plan");
    auto er = ensure(total, items.size(), nPk);
    if (er.has_error()) return er;

    for (size_t i = 0; i < items.size(); i++) {
        const size_t off = reinterpret_cast<size_t>(hDesc[i].data);
        if (items[i].bytes &&
            (rc = e2sar_hip_memcpy_async(ctx, dEvents + off, items[i].event, items[i].bytes, 0, nullptr)))
            return hip_error(rc, "event copy to device");
        auto &d = hDesc[i];
        d.data = dEvents + off;
        // lbEventNum = wall clock in microseconds, its low 8 bits random when the clock has
        // too little entropy there (cpp:707-719, addClockEntropy hpp:600-603); entropy 0 =>
        // random (cpp:727-728)
        d.lbTick = addEntropy ? ((detail::now_us() & ~uint64_t(0xFF)) | (rng() & 0xFFu)) : detail::now_us();
        d.eventNum = flags.ticksAsREEventNum ? d.lbTick : items[i].eventNum;   // cpp:723-724
        d.dataId = items[i].dataId;
        d.entropy = items[i].entropy ? items[i].entropy : (uint16_t)(rng() & 0xFFFF);
        d.reserved = 0;
    }
    if ((rc = e2sar_hip_memcpy_async(ctx, dDesc, hDesc.data(), items.size() * sizeof(e2sar_hip_seg_event), 0,
                                     nullptr)))
        return hip_error(rc, "event table copy");
    if ((rc = e2sar_hip_segment_batch(ctx, dDesc, (uint32_t)items.size(), maxPk, flags.lbHdrVersion,
                                      (uint32_t)maxPld, 1, dPkts, stride, dLens, nullptr)))
        return hip_error(rc, "segment_batch");
    // device -> host by the GPU's own stores into pinned memory (one copy_spans launch), not
    // by DMA: host->device copies (this Segmenter's events, a Reassembler's datagrams in the
    // same process) keep the DMA engines, which serialise when both directions share them
    // (tools/bench_hostpath.py: both directions at once 13.5 GiB/s each with DMA both ways,
    // 21.0 with device->host by kernel stores)
    const e2sar_hip_copy_span back[2] = {{dPkts, hPkts, (uint64_t)nPk * stride}, {dLens, hLens, (uint64_t)nPk * 4}};
    if ((rc = e2sar_hip_copy_spans(ctx, back, 2, nullptr)) || (rc = e2sar_hip_stream_sync(ctx, nullptr)))
        return hip_error(rc, "datagram copy to host");

    // one sendmmsg per event, round-robin over the sockets (cpp:404, 834-857)
    std::vector<mmsghdr> mv;
    std::vector<iovec> iv;
    for (size_t i = 0; i < items.size(); i++) {
        const uint32_t base = hDesc[i].pktBase;
        const uint32_t n = (uint32_t)e2sar_hip_num_packets(items[i].bytes, maxPld);
        const size_t s = rr++ % fds.size();
        mv.assign(n, mmsghdr{});
        iv.resize(n);
        for (uint32_t k = 0; k < n; k++) {
            iv[k].iov_base = hPkts + (size_t)(base + k) * stride;
            iv[k].iov_len = hLens[base + k];
            mv[k].msg_hdr.msg_iov = &iv[k];
            mv[k].msg_hdr.msg_iovlen = 1;
            if (!flags.connectedSocket) {
                mv[k].msg_hdr.msg_name = &dsts[s];
                mv[k].msg_hdr.msg_namelen = dstLen;
            }
        }
        // start-to-start pacing, as the reference's busy wait from the dispatch time
        // (cpp:401, 447-450): the next event may start interval after this one started
        if (flags.rateGbps > 0) {
            const auto now = std::chrono::steady_clock::now();
            if (paceNext > now) {
                if (paceNext - now > std::chrono::microseconds(200))
                    std::this_thread::sleep_until(paceNext - std::chrono::microseconds(100));
                while (std::chrono::steady_clock::now() < paceNext) {
                }
            } else {
                paceNext = now;   // behind schedule: no credit is banked
            }
            paceNext += std::chrono::nanoseconds((int64_t)((double)items[i].bytes * 8.0 / flags.rateGbps));
        }
        // at most sendChunk datagrams per call: the kernel hands a loopback or local
        // receiver's datagrams over when the call returns, and a whole event's worth in one
        // call (731 at MTU 1500) overruns its per-CPU backlog; short calls keep the sender
        // at the rate the receiving side drains
        static const uint32_t sendChunk = [] {
            const char *v = getenv("E2SAR_SEND_CHUNK");
            const unsigned long x = v ? strtoul(v, nullptr, 10) : 64ul;
            return (uint32_t)(x ? x : 0xFFFFFFFFul);
        }();
        uint32_t sent = 0;
        while (sent < n) {
            const int r = sendmmsg(fds[s], mv.data() + sent, std::min(n - sent, sendChunk), 0);
            if (r < 0) {
                if (errno == EINTR) continue;
                if (errno == EAGAIN || errno == ENOBUFS) {
                    std::this_thread::yield();
                    continue;
                }
                errCnt += n - sent;
                lastErrno = errno;
                lastErr = E2SARErrorc::SocketError;
                return E2SARErrorInfo{E2SARErrorc::SocketError, strerror(errno)};
            }
            sent += (uint32_t)r;
        }
        msgCnt += n;
    }
    return 0;
}

void Segmenter::Impl::threadBody()
{
    std::vector<Item> batch;
    while (true) {
        {
            std::unique_lock<std::mutex> lk(qMu);
            qCv.wait_for(lk, std::chrono::milliseconds(10), [&] { return stop.load() || !q.empty(); });
            if (q.empty()) {
                if (stop) return;
                continue;
            }
            batch.clear();
            size_t bytes = 0;
            while (!q.empty() && batch.size() < flags.maxBatchEvents &&
                   (batch.empty() || bytes + q.front().bytes <= flags.maxBatchBytes)) {
                bytes += q.front().bytes;
                batch.push_back(std::move(q.front()));
                q.pop_front();
            }
            inFlight = batch.size();
        }
        auto res = sendBatch(batch);
        if (res.has_error()) lastErr = res.error().code();
        for (auto &it : batch)
            if (it.cb) it.cb(it.cbArg);   // after the event's last datagram (cpp:436-438)
        {
            std::lock_guard<std::mutex> lk(qMu);
            inFlight = 0;
        }
        qEmptyCv.notify_all();
    }
}

// SyncThreadState::_open (e2sarDPSegmenter.cpp:282-337): a UDP socket to the URI's sync
// address, connected unless connectedSocket is false
result<int> Segmenter::Impl::syncOpen()
{
    auto sa = uri.get_syncAddr();
    if (sa.has_error()) return sa.error();
    const std::string &host = sa.value().first;
    const bool v6 = host.find(':') != std::string::npos;
    syncDst = sockaddr_storage{};
    int ok;
    if (v6) {
        auto *a = reinterpret_cast<sockaddr_in6 *>(&syncDst);
        a->sin6_family = AF_INET6;
        a->sin6_port = htons(sa.value().second);
        ok = inet_pton(AF_INET6, host.c_str(), &a->sin6_addr);
        syncDstLen = sizeof(sockaddr_in6);
    } else {
        auto *a = reinterpret_cast<sockaddr_in *>(&syncDst);
        a->sin_family = AF_INET;
        a->sin_port = htons(sa.value().second);
        ok = inet_pton(AF_INET, host.c_str(), &a->sin_addr);
        syncDstLen = sizeof(sockaddr_in);
    }
    if (ok != 1) return E2SARErrorInfo{E2SARErrorc::ParameterError, "bad sync address " + host};
    syncFd = socket(v6 ? AF_INET6 : AF_INET, SOCK_DGRAM, 0);
    if (syncFd < 0 ||
        (flags.connectedSocket && connect(syncFd, reinterpret_cast<sockaddr *>(&syncDst), syncDstLen) != 0)) {
        syncErrCnt++;
        syncLastErrno = errno;
        if (syncFd >= 0) close(syncFd);
        syncFd = -1;
        return E2SARErrorInfo{E2SARErrorc::SocketError, strerror(syncLastErrno.load())};
    }
    return 0;
}

// fillSyncHdr (hpp:583-591) + _send (cpp:345-373): the reported event number is the wall
// clock in microseconds (the LB tick the data path stamps), the rate a constant 1 MHz,
// the time the wall clock in nanoseconds
void Segmenter::Impl::syncSend()
{
    const uint64_t nowNs = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                               std::chrono::system_clock::now().time_since_epoch())
                               .count();
    SyncHdr hdr{};
    hdr.set(eventSrcId, detail::now_us(), 1000000u, nowNs);
    syncMsgCnt++;
    const ssize_t r = flags.connectedSocket
                          ? send(syncFd, &hdr, sizeof(hdr), 0)
                          : sendto(syncFd, &hdr, sizeof(hdr), 0, reinterpret_cast<sockaddr *>(&syncDst), syncDstLen);
    if (r < 0) {
        syncErrCnt++;
        syncLastErrno = errno;
    }
}

// SyncThreadState::_threadBody (cpp:242-280): one SyncHdr per syncPeriodMs, start to start
void Segmenter::Impl::syncBody()
{
    auto next = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(syncMu);
    while (!syncStop) {
        lk.unlock();
        syncSend();
        lk.lock();
        next += std::chrono::milliseconds(flags.syncPeriodMs);
        syncCv.wait_until(lk, next, [&] { return syncStop; });
    }
}

void Segmenter::Impl::syncHalt()
{
    {
        std::lock_guard<std::mutex> lk(syncMu);
        syncStop = true;
    }
    syncCv.notify_all();
    if (syncThread.joinable()) syncThread.join();
    if (syncFd >= 0) close(syncFd);     // _close (cpp:279, 339-343)
    syncFd = -1;
}

// cpp:160-191 (the Sync thread and its warm-up first, as there); sockets as in cpp:470-657
result<int> Segmenter::openAndStart() noexcept
{
    auto &m = *impl;
    if (m.started) return 0;
    auto addr = m.useV6 ? m.uri.get_dataAddrv6() : m.uri.get_dataAddrv4();
    if (addr.has_error()) return addr.error();
    if (m.flags.useCP && !m.syncThread.joinable()) {
        auto so = m.syncOpen();
        if (so.has_error())
            return E2SARErrorInfo{E2SARErrorc::SocketError, "Unable to open sync socket: " + so.error().message()};
        m.syncStop = false;
        m.syncThread = std::thread([&m] { m.syncBody(); });
        // a warm-up period of Sync packets and no data (cpp:174-175)
        std::this_thread::sleep_for(std::chrono::milliseconds(m.flags.warmUpMs));
    }
    std::uniform_int_distribution<int> portDist(10000, 65535);
    for (size_t i = 0; i < m.flags.numSendSockets; i++) {
        sockaddr_storage ss{};
        socklen_t sl;
        const uint16_t port = (uint16_t)(addr.value().second + (m.flags.multiPort ? i : 0));
        if (m.useV6) {
            auto *a = reinterpret_cast<sockaddr_in6 *>(&ss);
            a->sin6_family = AF_INET6;
            a->sin6_port = htons(port);
            if (inet_pton(AF_INET6, addr.value().first.c_str(), &a->sin6_addr) != 1)
                return E2SARErrorInfo{E2SARErrorc::ParameterError, "bad IPv6 data address"};
            sl = sizeof(sockaddr_in6);
        } else {
            auto *a = reinterpret_cast<sockaddr_in *>(&ss);
            a->sin_family = AF_INET;
            a->sin_port = htons(port);
            if (inet_pton(AF_INET, addr.value().first.c_str(), &a->sin_addr) != 1)
                return E2SARErrorInfo{E2SARErrorc::ParameterError, "bad IPv4 data address"};
            sl = sizeof(sockaddr_in);
        }
        const int fd = socket(m.useV6 ? AF_INET6 : AF_INET, SOCK_DGRAM, 0);
        if (fd < 0) return E2SARErrorInfo{E2SARErrorc::SocketError, strerror(errno)};
        setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &m.flags.sndSocketBufSize, sizeof(int));
        // random source port (hpp:237); fall back to an ephemeral one if taken
        for (int tries = 0; tries < 16; tries++) {
            sockaddr_storage src{};
            if (m.useV6) {
                auto *a = reinterpret_cast<sockaddr_in6 *>(&src);
                a->sin6_family = AF_INET6;
                a->sin6_port = htons((uint16_t)portDist(m.rng));
                a->sin6_addr = in6addr_any;
            } else {
                auto *a = reinterpret_cast<sockaddr_in *>(&src);
                a->sin_family = AF_INET;
                a->sin_port = htons((uint16_t)portDist(m.rng));
                a->sin_addr.s_addr = htonl(INADDR_ANY);
            }
            if (bind(fd, reinterpret_cast<sockaddr *>(&src), sl) == 0) break;
        }
        if (m.flags.connectedSocket && connect(fd, reinterpret_cast<sockaddr *>(&ss), sl) != 0) {
            close(fd);
            return E2SARErrorInfo{E2SARErrorc::SocketError, strerror(errno)};
        }
        m.fds.push_back(fd);
        m.dsts.push_back(ss);
        m.dstLen = sl;
    }
    m.stop = false;
    m.sendThread = std::thread([&m] { m.threadBody(); });
    m.started = true;
    return 0;
}

// cpp:901-917
result<int> Segmenter::sendEvent(uint8_t *event, size_t bytes, EventNum_t _eventNum, uint16_t _dataId,
                                 uint16_t entropy) noexcept
{
    auto &m = *impl;
    if (!m.started) return E2SARErrorInfo{E2SARErrorc::LogicError, "openAndStart() has not been called"};
    if (_eventNum != 0) m.userEventNum.exchange(_eventNum);
    std::vector<Impl::Item> one(1);
    one[0] = Impl::Item{event, bytes, m.userEventNum++, (uint16_t)(_dataId == 0 ? m.dataId : _dataId), entropy,
                        nullptr, std::any()};
    try {
        auto r = m.sendBatch(one);
        if (r.has_error()) return r.error();
    } catch (const std::exception &e) {
        return E2SARErrorInfo{E2SARErrorc::CaughtException, e.what()};
    }
    return 0;
}

// cpp:920-948
result<int> Segmenter::addToSendQueue(uint8_t *event, size_t bytes, EventNum_t _eventNum, uint16_t _dataId,
                                      uint16_t entropy, void (*callback)(std::any), std::any cbArg) noexcept
{
    auto &m = *impl;
    try {
        std::lock_guard<std::mutex> lk(m.qMu);
        bool accepted;
        const EventNum_t num = detail::take_send_number(m.userEventNum, _eventNum, m.q.size(), Impl::kQueueCap, &accepted);
        if (!accepted)
            return E2SARErrorInfo{E2SARErrorc::MemoryError, "Send queue is temporarily full, try again later"};
        m.q.push_back(Impl::Item{event, bytes, num, (uint16_t)(_dataId == 0 ? m.dataId : _dataId),
                                 entropy, callback, std::move(cbArg)});
    } catch (const std::exception &e) {
        return E2SARErrorInfo{E2SARErrorc::CaughtException, e.what()};
    }
    m.qCv.notify_one();
    return 0;
}

const Segmenter::ReportedStats Segmenter::getSendStats() const noexcept
{
    return ReportedStats{impl->msgCnt.load(), impl->errCnt.load(), impl->lastErrno.load(), impl->lastErr.load()};
}

const Segmenter::ReportedStats Segmenter::getSyncStats() const noexcept
{
    return ReportedStats{impl->syncMsgCnt.load(), impl->syncErrCnt.load(), impl->syncLastErrno.load(),
                         E2SARErrorc::NoError};
}

const std::string Segmenter::getIntf() const noexcept { return impl->iface; }
uint16_t Segmenter::getMTU() const noexcept { return impl->mtu; }
size_t Segmenter::getMaxPldLen() const noexcept { return impl->maxPld; }
bool Segmenter::isUsingIPv6() const noexcept { return impl->useV6; }

// hpp:537-552: drain the queue, then stop the send thread
void Segmenter::stopThreads()
{
    auto &m = *impl;
    m.syncHalt();
    if (!m.started) return;
    {
        std::unique_lock<std::mutex> lk(m.qMu);
        m.qEmptyCv.wait(lk, [&] { return m.q.empty() && m.inFlight == 0; });
    }
    m.stop = true;
    m.qCv.notify_all();
    if (m.sendThread.joinable()) m.sendThread.join();
    m.started = false;
}

}  // namespace e2sar
