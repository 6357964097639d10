// reassembler.cpp -- e2sar::Reassembler over the gfx950 reassembly kernel.
//
// Reference: N receive threads, each owning a set of UDP ports, run the per-datagram body
// (e2sarDPReassembler.cpp:293-433) -- malloc, recvfrom, header checks, map lookup, memcpy
// -- one datagram at a time; a GC thread drops stale events (cpp:236-291).
// Here the receive threads only fill pinned datagram batches with recvmmsg (a slot of
// recvStride bytes per datagram); one device thread pipelines the batches through HBM:
// the host->device copy of batch b+1 runs on a copy stream beside the reassembly kernel of
// batch b (two device datagram buffers), a host batch goes back to the receive threads as
// soon as its copy has landed, and the events batch b completed leave the device arena in
// ONE gather launch into pinned staging, from which they are copied into the new[] buffers
// that getEvent/recvEvent hand over.  Lost-event records are drained the same way; the
// device GC pass runs every eventTimeout_ms; the table and arena are recycled or compacted
// when either passes half full.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <new>
#include <set>
#include <thread>

#include "host_common.hpp"

namespace e2sar {

using detail::hip_error;

struct Reassembler::Impl {
    EjfatURI uri;
    ReassemblerFlags flags;
    std::vector<int> cores;
    std::string dataIP;
    bool v6 = false;
    uint16_t dataPort;
    int portRange;
    size_t numRecvThreads;
    size_t numRecvPorts;
    std::vector<std::vector<uint16_t>> threadsToPorts;

    // device: the compute stream (the context's) and a copy stream; two device datagram
    // buffers so batch b+1 is copied in while batch b is reassembled
    e2sar_hip_ctx *ctx = nullptr;
    void *stream = nullptr;
    void *copyStream = nullptr;
    e2sar_hip_reas *reas = nullptr;
    struct DevSet {
        uint8_t *pkts = nullptr;
        uint32_t *lens = nullptr;
        void *h2dDone = nullptr;        // recorded on the copy stream after the batch's copy
    };
    DevSet sets[2];
    void *gatherDone = nullptr;         // recorded on the compute stream after a drain's gather
    uint8_t *stage = nullptr;           // pinned staging for completed events
    size_t stageBytes = 0;
    std::vector<size_t> stageOffs;      // staging offsets of the records of the gather in flight
    std::atomic<uint64_t> upkeeps{0};   // recycles + compactions done
    std::vector<e2sar_hip_event_rec> recs;
    std::vector<e2sar_hip_lost_rec> lrecs;

    // datagram batches (pinned)
    struct Batch {
        uint8_t *pkts = nullptr;
        uint32_t *lens = nullptr;
        uint32_t n = 0;
    };
    std::vector<Batch> batches;
    std::mutex bMu;
    std::condition_variable bFreeCv, bFullCv;
    std::deque<Batch *> freeB, fullB;

    // event queue (hpp:126-127: unbounded, see gatherFinish) and lost events (hpp:102-122, 262-279)
    struct Ev {
        uint8_t *event;
        size_t bytes;
        EventNum_t eventNum;
        uint16_t dataId;
    };
    std::mutex eMu;
    std::condition_variable eCv;
    std::deque<Ev> evq;
    std::mutex lMu;
    std::deque<std::tuple<EventNum_t, uint16_t, size_t>> lostq;
    std::set<std::pair<EventNum_t, uint16_t>> lostSeen;

    // host-side counters
    std::atomic<uint64_t> hostEnqueueLoss{0}, hostReassemblyLoss{0};
    std::atomic<int> lastErrno{0}, dataErrCnt{0};
    std::atomic<E2SARErrorc> lastErr{E2SARErrorc::NoError};
    std::map<uint16_t, std::atomic<size_t> *> perPort;
    std::vector<std::unique_ptr<std::atomic<size_t>>> perPortStore;

    std::vector<std::thread> recvThreads;
    std::thread devThread;
    std::atomic<bool> stop{false};
    std::atomic<int> recvActive{0};
    bool started = false;
    e2sar_hip_reas_stats lastStats{};
    std::mutex sMu;

    Impl(const EjfatURI &u, const ReassemblerFlags &f) : uri(u), flags(f) {}
    ~Impl();
    void setup(size_t nThreads);
    void recvBody(size_t t, std::vector<int> fds, std::vector<uint16_t> ports);
    void devBody();
    void drainLost();
    uint32_t gatherLaunch(uint32_t first, uint32_t n, uint8_t *arena);
    void gatherFinish(uint32_t first, uint32_t upto);
    bool needsUpkeep(const e2sar_hip_reas_stats &st) const;
    void upkeep(const e2sar_hip_reas_stats &st);
    Batch *takeFree();
    Batch *takeFull(bool wait);
    void giveBack(Batch *b);
};

Reassembler::Impl::~Impl()
{
    if (ctx) {
        e2sar_hip_stream_sync(ctx, stream);
        e2sar_hip_stream_sync(ctx, copyStream);
    }
    for (auto &b : batches) {
        if (b.pkts) e2sar_hip_host_free(b.pkts);
        if (b.lens) e2sar_hip_host_free(b.lens);
    }
    if (stage) e2sar_hip_host_free(stage);
    if (reas) e2sar_hip_reas_destroy(reas);
    if (ctx) {
        for (auto &d : sets) {
            if (d.pkts) e2sar_hip_device_free(ctx, d.pkts);
            if (d.lens) e2sar_hip_device_free(ctx, d.lens);
            e2sar_hip_event_destroy(d.h2dDone);
        }
        e2sar_hip_event_destroy(gatherDone);
        e2sar_hip_ctx_destroy(ctx);
    }
    if (stream) e2sar_hip_stream_destroy(stream);
    if (copyStream) e2sar_hip_stream_destroy(copyStream);
    std::lock_guard<std::mutex> lk(eMu);
    for (auto &e : evq) delete[] e.event;
}

// ctor body: port range and thread/port assignment (cpp:37-181, hpp:308-318)
void Reassembler::Impl::setup(size_t nThreads)
{
    numRecvThreads = nThreads;
    portRange = flags.portRange != -1 ? flags.portRange : get_PortRange((int)nThreads);
    numRecvPorts = (size_t)(portRange > 0 ? 2 << (portRange - 1) : 1);
    if (numRecvThreads > 128) throw E2SARException("Too many reassembly threads requested, limit 128");
    if (numRecvThreads == 0) throw E2SARException("At least one receive thread is required");
    if (portRange < 0 || portRange > 14) throw E2SARException("Port range out of bounds: [0, 14]");
    if (flags.recvStride % 16 || flags.recvStride < 48) throw E2SARException("recvStride must be a multiple of 16, >= 48");
    threadsToPorts.assign(numRecvThreads, {});
    for (size_t i = 0; i < numRecvPorts;)
        for (size_t j = 0; i < numRecvPorts && j < numRecvThreads; i++, j++)
            threadsToPorts[j].push_back((uint16_t)(dataPort + i));
    for (size_t i = 0; i < numRecvPorts; i++) {
        perPortStore.emplace_back(new std::atomic<size_t>(0));
        perPort[(uint16_t)(dataPort + i)] = perPortStore.back().get();
    }

    int rc = e2sar_hip_stream_create(flags.gpuDevice, &stream);
    if (rc == 0) rc = e2sar_hip_stream_create(flags.gpuDevice, &copyStream);
    if (rc == 0) rc = e2sar_hip_ctx_create(flags.gpuDevice, stream, &ctx);
    e2sar_hip_reas_config cfg{};
    cfg.withLBHeader = flags.withLBHeader ? 1 : 0;
    cfg.tableSlots = flags.tableSlots;
    cfg.queueCapacity = (uint32_t)std::max<size_t>(4096, flags.recvBatch);
    cfg.lostCapacity = 4096;
    cfg.arenaBytes = flags.arenaBytes;
    cfg.flags = E2SAR_HIP_REAS_COMPACTABLE | (flags.referenceOrder ? E2SAR_HIP_REAS_REFERENCE_ORDER : 0u);
    if (rc == 0) rc = e2sar_hip_reas_create(ctx, &cfg, &reas);
    for (auto &d : sets) {
        if (rc == 0) rc = e2sar_hip_device_alloc(ctx, flags.recvBatch * flags.recvStride, reinterpret_cast<void **>(&d.pkts));
        if (rc == 0) rc = e2sar_hip_device_alloc(ctx, flags.recvBatch * 4, reinterpret_cast<void **>(&d.lens));
        if (rc == 0) rc = e2sar_hip_event_create(ctx, &d.h2dDone);
    }
    if (rc == 0) rc = e2sar_hip_event_create(ctx, &gatherDone);
    stageBytes = std::max<size_t>(size_t(64) << 20, 2 * flags.recvBatch * flags.recvStride);
    if (rc == 0) rc = e2sar_hip_host_alloc(stageBytes, reinterpret_cast<void **>(&stage));
    // host batches: two per receive thread being filled / queued, two on their way to the
    // device, and slack so a receive thread never waits for one while the device thread
    // still holds batches whose copies are done but not yet handed back (MTU 9000 loopback
    // lost datagrams with 4: 0.1 s of waiting for a free batch)
    const size_t nb = 2 * numRecvThreads + 6;
    batches.resize(nb);
    for (auto &b : batches) {
        if (rc == 0) rc = e2sar_hip_host_alloc(flags.recvBatch * flags.recvStride, reinterpret_cast<void **>(&b.pkts));
        if (rc == 0) rc = e2sar_hip_host_alloc(flags.recvBatch * 4, reinterpret_cast<void **>(&b.lens));
        freeB.push_back(&b);
    }
    if (rc) throw E2SARException(std::string("Unable to set up the GPU reassembler: ") + e2sar_hip_last_error());
    recs.resize(cfg.queueCapacity);
    lrecs.resize(cfg.lostCapacity);
}

Reassembler::Reassembler(const EjfatURI &uri, const std::string &data_ip, uint16_t starting_port,
                         std::vector<int> cpuCoreList, const ReassemblerFlags &rflags)
    : impl(new Impl(uri, rflags))
{
    impl->dataIP = data_ip;
    impl->v6 = data_ip.find(':') != std::string::npos;
    impl->dataPort = starting_port;
    impl->cores = cpuCoreList;
    impl->setup(cpuCoreList.size());
}

Reassembler::Reassembler(const EjfatURI &uri, const std::string &data_ip, uint16_t starting_port,
                         size_t numRecvThreads, const ReassemblerFlags &rflags)
    : impl(new Impl(uri, rflags))
{
    impl->dataIP = data_ip;
    impl->v6 = data_ip.find(':') != std::string::npos;
    impl->dataPort = starting_port;
    impl->setup(numRecvThreads);
}

Reassembler::Reassembler(const EjfatURI &uri, uint16_t starting_port, std::vector<int> cpuCoreList,
                         const ReassemblerFlags &rflags, bool v6)
    : impl(new Impl(uri, rflags))
{
    impl->dataIP = v6 ? "::" : "0.0.0.0";
    impl->v6 = v6;
    impl->dataPort = starting_port;
    impl->cores = cpuCoreList;
    impl->setup(cpuCoreList.size());
}

Reassembler::Reassembler(const EjfatURI &uri, uint16_t starting_port, size_t numRecvThreads,
                         const ReassemblerFlags &rflags, bool v6)
    : impl(new Impl(uri, rflags))
{
    impl->dataIP = v6 ? "::" : "0.0.0.0";
    impl->v6 = v6;
    impl->dataPort = starting_port;
    impl->setup(numRecvThreads);
}

Reassembler::~Reassembler() { stopThreads(); }

Reassembler::Impl::Batch *Reassembler::Impl::takeFree()
{
    std::unique_lock<std::mutex> lk(bMu);
    while (freeB.empty() && !stop) bFreeCv.wait_for(lk, std::chrono::milliseconds(10));
    if (freeB.empty()) return nullptr;
    Batch *b = freeB.front();
    freeB.pop_front();
    b->n = 0;
    return b;
}

// The receive loop: select/recvfrom (cpp:293-333) become poll + recvmmsg into a batch.
void Reassembler::Impl::recvBody(size_t, std::vector<int> fds, std::vector<uint16_t> ports)
{
    std::vector<pollfd> pf(fds.size());
    for (size_t i = 0; i < fds.size(); i++) pf[i] = pollfd{fds[i], POLLIN, 0};
    const size_t cap = flags.recvBatch;
    const size_t S = flags.recvStride;
    std::vector<mmsghdr> mv(cap);
    std::vector<iovec> iv(cap);
    // the message vector of a batch points at its slots; built once per batch (recvmmsg only
    // writes msg_len / msg_flags back), so a call that returns few datagrams costs no setup
    const Batch *vecFor = nullptr;
    auto vectorFor = [&](const Batch *x) {
        if (vecFor == x) return;
        for (size_t k = 0; k < cap; k++) {
            iv[k].iov_base = x->pkts + k * S;
            iv[k].iov_len = S;
            mv[k].msg_hdr = msghdr{};
            mv[k].msg_hdr.msg_iov = &iv[k];
            mv[k].msg_hdr.msg_iovlen = 1;
        }
        vecFor = x;
    };
    // E2SAR_RECV_PROFILE=1: where the receive thread's time goes (stderr at exit)
    static const bool prof = getenv("E2SAR_RECV_PROFILE") != nullptr;
    uint64_t tPoll = 0, tRecv = 0, tFree = 0, nCalls = 0, nDg = 0, nFlush = 0, tLastDg = 0, t0 = detail::now_us();
    static const uint64_t spinUs = [] {
        const char *v = getenv("E2SAR_RECV_SPIN_US");
        return v ? (uint64_t)strtoull(v, nullptr, 10) : 200ull;
    }();
    uint64_t lastData = 0;
    Batch *b = takeFree();
    uint64_t firstUs = 0;
    auto flush = [&]() {
        if (!b || b->n == 0) return;
        {
            std::lock_guard<std::mutex> lk(bMu);
            fullB.push_back(b);
        }
        bFullCv.notify_one();
        const uint64_t a = prof ? detail::now_us() : 0;
        b = takeFree();
        if (prof) tFree += detail::now_us() - a, nFlush++;
        firstUs = 0;
    };
    while (!stop) {
        if (!b) {
            b = takeFree();
            if (!b) continue;
        }
        const int timeout = (b->n > 0) ? std::max(1, flags.batchTimeout_us / 1000) : 10;   // 10 ms like sleep_tv
        // while datagrams keep coming, stay awake and poll the sockets with non-blocking
        // recvmmsg for up to spinUs after the last one: a sleeping receiver costs the
        // sending side one wakeup per datagram (loopback: half the datagram rate)
        int pr;
        if (lastData && detail::now_us() - lastData < spinUs) {
            for (auto &p : pf) p.revents = POLLIN;
            pr = (int)pf.size();
        } else {
            const uint64_t pa = prof ? detail::now_us() : 0;
            pr = poll(pf.data(), pf.size(), timeout);
            if (prof) tPoll += detail::now_us() - pa;
        }
        if (pr < 0) {
            if (errno != EINTR) {
                dataErrCnt++;
                lastErrno = errno;
            }
            continue;
        }
        for (size_t i = 0; i < pf.size() && b; i++) {
            if (!(pf[i].revents & POLLIN)) continue;
            while (b && b->n < cap) {
                const size_t room = cap - b->n;
                vectorFor(b);
                mmsghdr *const m = mv.data() + b->n;
                const uint64_t ra = prof ? detail::now_us() : 0;
                const int r = recvmmsg(fds[i], m, (unsigned)room, MSG_DONTWAIT, nullptr);
                if (prof) {
                    tRecv += detail::now_us() - ra, nCalls++, nDg += r > 0 ? (uint64_t)r : 0u;
                    if (r > 0) tLastDg = detail::now_us() - t0;
                }
                if (r < 0) {
                    if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
                        dataErrCnt++;
                        lastErrno = errno;
                    }
                    break;
                }
                for (int k = 0; k < r; k++) {
                    uint32_t len = m[k].msg_len;
                    if (m[k].msg_hdr.msg_flags & MSG_TRUNC) len = (uint32_t)S + 1;   // device: dataErrCnt
                    b->lens[b->n + k] = len;
                }
                perPort[ports[i]]->fetch_add((size_t)r);
                if (r > 0) lastData = detail::now_us();
                if (b->n == 0 && r > 0) firstUs = detail::now_us();
                b->n += (uint32_t)r;
                if (b->n == cap) flush();
                if (r < (int)room) break;
            }
        }
        // (A/B, dropped: flushing a partial batch only while the device thread waits for one
        // lost jumbo datagrams at MTU 9000 -- the batch then grows to 9 MB behind a busy
        // device -- and gained nothing at 1500)
        if (b && b->n > 0 && detail::now_us() - firstUs >= (uint64_t)flags.batchTimeout_us) flush();
    }
    if (prof)
        fprintf(stderr, "recv thread: %.3f s, poll %.3f s, recvmmsg %.3f s (%llu calls, %llu datagrams), "
                        "waiting for a free batch %.3f s (%llu batches), last datagram at %.3f s\n",
                (detail::now_us() - t0) * 1e-6, tPoll * 1e-6, tRecv * 1e-6, (unsigned long long)nCalls,
                (unsigned long long)nDg, tFree * 1e-6, (unsigned long long)nFlush, tLastDg * 1e-6);
    if (b) {
        if (b->n) {
            std::lock_guard<std::mutex> lk(bMu);
            fullB.push_back(b);
        } else {
            std::lock_guard<std::mutex> lk(bMu);
            freeB.push_back(b);
        }
        bFullCv.notify_one();
    }
}

Reassembler::Impl::Batch *Reassembler::Impl::takeFull(bool wait)
{
    std::unique_lock<std::mutex> lk(bMu);
    if (wait) bFullCv.wait_for(lk, std::chrono::milliseconds(10), [&] { return stop.load() || !fullB.empty(); });
    if (fullB.empty()) return nullptr;
    Batch *b = fullB.front();
    fullB.pop_front();
    return b;
}

void Reassembler::Impl::giveBack(Batch *b)
{
    {
        std::lock_guard<std::mutex> lk(bMu);
        freeB.push_back(b);
    }
    bFreeCv.notify_all();
}

// Completed records recs[first, n) (already polled; their bytes in `arena`) -> pinned
// staging, as many as fit, in one gather launch (e2sar_hip_copy_spans) on the compute
// stream, so it runs ahead of any later kernel or recycle that could overwrite them.
// Returns the index past the last record launched; gatherFinish waits for that launch and
// copies the events into the new[] buffers the caller will own (bin/e2sar_perf.cpp:299).
uint32_t Reassembler::Impl::gatherLaunch(uint32_t first, uint32_t n, uint8_t *arena)
{
    stageOffs.clear();
    std::vector<e2sar_hip_copy_span> spans;
    size_t used = 0;
    uint32_t i = first;
    for (; i < n; i++) {
        const size_t b = recs[i].bytes;
        const size_t need = (b + 63) & ~(size_t)63;
        if (need > stageBytes && i == first) {          // larger than all of the staging: grow it
            e2sar_hip_stream_sync(ctx, stream);
            e2sar_hip_host_free(stage);
            stage = nullptr;
            stageBytes = 0;
            if (e2sar_hip_host_alloc(need, reinterpret_cast<void **>(&stage)) != 0) {
                lastErr = E2SARErrorc::MemoryError;
                return n;
            }
            stageBytes = need;
        }
        if (used + need > stageBytes) break;
        stageOffs.push_back(used);
        if (b) spans.push_back(e2sar_hip_copy_span{arena + recs[i].arenaOffset, stage + used, b});
        used += need;
    }
    int rc = e2sar_hip_copy_spans(ctx, spans.data(), (uint32_t)spans.size(), stream);
    if (rc == 0) rc = e2sar_hip_event_record(ctx, gatherDone, stream);
    if (rc) lastErr = E2SARErrorc::SystemError;
    return i;
}

void Reassembler::Impl::gatherFinish(uint32_t first, uint32_t upto)
{
    if (upto <= first) return;
    if (e2sar_hip_event_sync(gatherDone) != 0 || stageOffs.size() != upto - first) {
        lastErr = E2SARErrorc::SystemError;
        return;
    }
    // The reference's eventQueue (hpp:126-127) is a boost::lockfree::queue without
    // fixed_sized: QSIZE only pre-sizes its node pool and push() allocates past it, so an
    // enqueue fails (hpp:138-144 -> enqueueLoss, cpp:413-421) only when allocation does.
    // The queue here is unbounded the same way; a failed allocation is the only loss.
    auto lose = [this](EventNum_t eventNum, uint16_t dataId) {
        hostEnqueueLoss++;
        std::lock_guard<std::mutex> l2(lMu);
        if (lostSeen.insert({eventNum, dataId}).second) lostq.emplace_back(eventNum, dataId, 0);
    };
    std::vector<Ev> ready;
    ready.reserve(upto - first);
    for (uint32_t k = first; k < upto; k++) {
        const auto &r = recs[k];
        auto *buf = new (std::nothrow) uint8_t[r.bytes ? r.bytes : 1];
        if (!buf) {
            lose(r.eventNum, r.dataId);
            continue;
        }
        if (r.bytes) memcpy(buf, stage + stageOffs[k - first], r.bytes);
        ready.push_back(Ev{buf, r.bytes, r.eventNum, r.dataId});
    }
    {
        std::lock_guard<std::mutex> lk(eMu);
        for (auto &e : ready) {
            try {
                evq.push_back(e);
            } catch (const std::bad_alloc &) {
                lose(e.eventNum, e.dataId);
                delete[] e.event;
            }
        }
    }
    eCv.notify_all();
}

void Reassembler::Impl::drainLost()
{
    uint32_t nl = 0;
    if (e2sar_hip_reas_lost_poll(reas, lrecs.data(), (uint32_t)lrecs.size(), &nl) == 0 && nl) {
        std::lock_guard<std::mutex> l2(lMu);
        for (uint32_t i = 0; i < nl; i++) {   // logLostEvent dedupe (hpp:266-269)
            const auto &l = lrecs[i];
            if (lostSeen.insert({l.eventNum, l.dataId}).second) lostq.emplace_back(l.eventNum, l.dataId, l.numFragments);
        }
    }
}

// Recycle or compact once the arena or the table is half used.  Completed and timed-out
// slots keep their table entries until then, so with small events and a steady stream
// the table fills long before the arena; compaction keeps only the events in progress.
// It is skipped when it would not free at least half of the table (most slots live).
// Runs with the device idle and every completed record polled and gathered.
bool Reassembler::Impl::needsUpkeep(const e2sar_hip_reas_stats &st) const
{
    if (st.completedPending != 0) return false;
    const bool arenaHalf = st.arenaUsed > flags.arenaBytes / 2;
    const bool tableHalf = st.tableUsed > flags.tableSlots / 2 &&
                           st.tableUsed > 2 * (uint64_t)std::max<int64_t>(st.inProgress, 0);
    return arenaHalf || tableHalf;
}

void Reassembler::Impl::upkeep(const e2sar_hip_reas_stats &st)
{
    const int rc = st.inProgress == 0 ? e2sar_hip_reas_recycle(reas, 0, nullptr) : e2sar_hip_reas_compact(reas, nullptr);
    if (rc) lastErr = static_cast<E2SARErrorc>(-rc);
    else upkeeps++;
}

// The device thread.  Per batch b (two device buffers, sets[b % 2]):
//   copy b+1 in (copy stream, beside kernel b) -> poll b (waits for kernel b and the copy)
//   -> hand b+1's host batch back -> stats (device idle) -> gather b's events (compute
//   stream) -> [GC pass / recycle / compact, before any later kernel] -> kernel b+1
//   (after the copy's event) -> host copies of b's events while kernel b+1 runs.
void Reassembler::Impl::devBody()
{
    uint64_t lastGc = detail::steady_ms();
    const uint32_t stride = (uint32_t)flags.recvStride;
    bool kernelInFlight = false;       // a launched batch whose results are not yet drained
    int cur = 0;                       // device set of the next copy
    static const bool prof = getenv("E2SAR_RECV_PROFILE") != nullptr;
    uint64_t pT0 = detail::now_us(), pWait = 0, pPoll = 0, pGather = 0, pUpkeep = 0, pLaunch = 0, pCycles = 0,
             pBatches = 0, pDg = 0, pEvents = 0, pLastEv = 0;
    auto tick = [&]() { return prof ? detail::now_us() : 0; };
    while (true) {
        uint64_t ta = tick();
        Batch *b = takeFull(!kernelInFlight);
        if (prof) pWait += tick() - ta, pCycles++, pBatches += b ? 1 : 0, pDg += b ? b->n : 0;
        if (!b && !kernelInFlight && stop && recvActive.load() == 0) {
            std::lock_guard<std::mutex> lk(bMu);
            if (fullB.empty()) break;
        }
        DevSet &d = sets[cur];
        uint32_t bn = 0;
        uint64_t bnow = 0;
        if (b) {
            bn = b->n;
            bnow = detail::steady_ms();
            int rc = e2sar_hip_memcpy_async(ctx, d.pkts, b->pkts, (size_t)b->n * stride, 0, copyStream);
            if (rc == 0) rc = e2sar_hip_memcpy_async(ctx, d.lens, b->lens, (size_t)b->n * 4, 0, copyStream);
            if (rc == 0) rc = e2sar_hip_event_record(ctx, d.h2dDone, copyStream);
            if (rc) lastErr = static_cast<E2SARErrorc>(-rc);
        }
        uint32_t n = 0;
        ta = tick();
        if (e2sar_hip_reas_poll(reas, recs.data(), (uint32_t)recs.size(), &n) != 0) lastErr = E2SARErrorc::SystemError;
        if (prof) pPoll += tick() - ta, pEvents += n, pLastEv = n ? tick() - pT0 : pLastEv;
        if (b) giveBack(b);                                   // its bytes are on the device now
        kernelInFlight = false;
        e2sar_hip_reas_stats st{};
        const bool haveStats = e2sar_hip_reas_get_stats(reas, &st) == 0;
        if (haveStats) {
            std::lock_guard<std::mutex> lk(sMu);
            lastStats = st;
        }
        uint8_t *arena = e2sar_hip_reas_arena(reas);
        uint32_t upto = n ? gatherLaunch(0, n, arena) : 0;
        const uint64_t now = detail::steady_ms();
        const bool gcDue = now - lastGc >= (uint64_t)flags.eventTimeout_ms;
        const bool upkeepDue = haveStats && needsUpkeep(st);
        uint32_t done = 0;
        ta = tick();
        if (gcDue || upkeepDue) {
            // every completed event leaves the arena before the GC pass, a recycle or a compaction
            for (gatherFinish(0, upto), done = upto; done < n; done = upto) {
                upto = gatherLaunch(done, n, arena);
                gatherFinish(done, upto);
            }
            if (gcDue) {                              // GC thread period (cpp:252-283)
                e2sar_hip_reas_gc(reas, now, (uint64_t)flags.eventTimeout_ms, nullptr);
                lastGc = now;
                drainLost();
            }
            if (upkeepDue) upkeep(st);
        }
        if (prof) pUpkeep += tick() - ta;
        ta = tick();
        if (b) {
            int rc = e2sar_hip_stream_wait_event(ctx, nullptr, d.h2dDone);
            if (rc == 0) rc = e2sar_hip_reassemble_batch(reas, d.pkts, stride, d.lens, bn, bnow, nullptr);
            if (rc) lastErr = static_cast<E2SARErrorc>(-rc);
            else kernelInFlight = true;
            cur ^= 1;
        }
        if (prof) pLaunch += tick() - ta;
        ta = tick();
        if (done < n) {                                // while that kernel runs
            gatherFinish(done, upto);
            for (done = upto; done < n; done = upto) {
                upto = gatherLaunch(done, n, arena);
                gatherFinish(done, upto);
            }
        }
        if (prof) pGather += tick() - ta;
    }
    if (prof)
        fprintf(stderr, "device thread: %.3f s, %llu cycles (%llu batches, %llu datagrams, %llu events), waiting %.3f s, "
                        "poll %.3f s, upkeep/GC %.3f s, copy+launch %.3f s, gather %.3f s, last event at %.3f s\n",
                (detail::now_us() - pT0) * 1e-6, (unsigned long long)pCycles, (unsigned long long)pBatches,
                (unsigned long long)pDg, (unsigned long long)pEvents, pWait * 1e-6, pPoll * 1e-6, pUpkeep * 1e-6,
                pLaunch * 1e-6, pGather * 1e-6, pLastEv * 1e-6);
    uint32_t n = 0;
    if (e2sar_hip_reas_poll(reas, recs.data(), (uint32_t)recs.size(), &n) == 0 && n) {
        uint8_t *arena = e2sar_hip_reas_arena(reas);
        for (uint32_t done = 0, upto; done < n; done = upto) {
            upto = gatherLaunch(done, n, arena);
            gatherFinish(done, upto);
        }
    }
    drainLost();
}

result<int> Reassembler::registerWorker(const std::string &) noexcept
{
    if (impl->flags.useCP) return E2SARErrorInfo{E2SARErrorc::LogicError, "no control plane on this data path"};
    return 0;   // cpp:603-612 with useCP == false
}

result<int> Reassembler::deregisterWorker() noexcept { return 0; }

// cpp:184-234 and socket open cpp:435-510
result<int> Reassembler::openAndStart() noexcept
{
    auto &m = *impl;
    if (m.started) return 0;
    std::vector<std::vector<int>> tfds(m.numRecvThreads);
    for (size_t t = 0; t < m.numRecvThreads; t++) {
        for (uint16_t port : m.threadsToPorts[t]) {
            const int fd = socket(m.v6 ? AF_INET6 : AF_INET, SOCK_DGRAM, 0);
            if (fd < 0) return E2SARErrorInfo{E2SARErrorc::SocketError, strerror(errno)};
            setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &m.flags.rcvSocketBufSize, sizeof(int));
            const int one = 1;
            setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
            sockaddr_storage ss{};
            socklen_t sl;
            if (m.v6) {
                auto *a = reinterpret_cast<sockaddr_in6 *>(&ss);
                a->sin6_family = AF_INET6;
                a->sin6_port = htons(port);
                inet_pton(AF_INET6, m.dataIP.c_str(), &a->sin6_addr);
                sl = sizeof(sockaddr_in6);
            } else {
                auto *a = reinterpret_cast<sockaddr_in *>(&ss);
                a->sin_family = AF_INET;
                a->sin_port = htons(port);
                inet_pton(AF_INET, m.dataIP.c_str(), &a->sin_addr);
                sl = sizeof(sockaddr_in);
            }
            if (bind(fd, reinterpret_cast<sockaddr *>(&ss), sl) != 0) {
                const std::string err = strerror(errno);
                close(fd);
                for (auto &v : tfds)
                    for (int f : v) close(f);
                return E2SARErrorInfo{E2SARErrorc::SocketError, "bind port " + std::to_string(port) + ": " + err};
            }
            tfds[t].push_back(fd);
        }
    }
    m.stop = false;
    m.recvActive = (int)m.numRecvThreads;
    for (size_t t = 0; t < m.numRecvThreads; t++)
        m.recvThreads.emplace_back([&m, t, fds = tfds[t]] {
            m.recvBody(t, fds, m.threadsToPorts[t]);
            for (int f : fds) close(f);
            m.recvActive--;
            m.bFullCv.notify_one();
        });
    m.devThread = std::thread([&m] { m.devBody(); });
    m.started = true;
    return 0;
}

// cpp:626-641
result<int> Reassembler::getEvent(uint8_t **event, size_t *bytes, EventNum_t *eventNum, uint16_t *dataId) noexcept
{
    auto &m = *impl;
    std::lock_guard<std::mutex> lk(m.eMu);
    if (m.evq.empty()) return -1;
    const auto e = m.evq.front();
    m.evq.pop_front();
    *event = e.event;
    *bytes = e.bytes;
    *eventNum = e.eventNum;
    *dataId = e.dataId;
    return 0;
}

// cpp:643-676: wait in 10 ms slices; wait_ms == 0 waits until stopThreads()
result<int> Reassembler::recvEvent(uint8_t **event, size_t *bytes, EventNum_t *eventNum, uint16_t *dataId,
                                   uint64_t wait_ms) noexcept
{
    auto &m = *impl;
    const auto t0 = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(m.eMu);
    while (m.evq.empty()) {
        if (m.stop) return -1;
        m.eCv.wait_for(lk, std::chrono::milliseconds(10));
        if (wait_ms && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(wait_ms) && m.evq.empty())
            return -1;
    }
    const auto e = m.evq.front();
    m.evq.pop_front();
    *event = e.event;
    *bytes = e.bytes;
    *eventNum = e.eventNum;
    *dataId = e.dataId;
    return 0;
}

const Reassembler::ReportedStats Reassembler::getStats() const noexcept
{
    auto &m = *impl;
    e2sar_hip_reas_stats st{};
    if (!m.started || e2sar_hip_reas_get_stats(m.reas, &st) != 0) {
        std::lock_guard<std::mutex> lk(m.sMu);
        st = m.lastStats;
    }
    ReportedStats r{};
    r.enqueueLoss = st.enqueueLoss + m.hostEnqueueLoss.load();
    r.reassemblyLoss = st.reassemblyLoss + m.hostReassemblyLoss.load();
    r.eventSuccess = st.eventSuccess;
    r.lastErrno = m.lastErrno.load();
    r.grpcErrCnt = 0;
    r.dataErrCnt = m.dataErrCnt.load() + (int)st.dataErrCnt;
    r.lastE2SARError = m.lastErr.load();
    r.totalPackets = st.totalPackets;
    r.totalBytes = st.totalBytes;
    r.badHeaderDiscards = st.badHeaderDiscards;
    return r;
}

result<std::tuple<EventNum_t, uint16_t, size_t>> Reassembler::get_LostEvent() noexcept
{
    auto &m = *impl;
    std::lock_guard<std::mutex> lk(m.lMu);
    if (m.lostq.empty()) return E2SARErrorInfo{E2SARErrorc::NotFound, "Lost event queue is empty"};
    auto t = m.lostq.front();
    m.lostq.pop_front();
    return t;
}

result<std::list<std::pair<uint16_t, size_t>>> Reassembler::get_FDStats() noexcept
{
    auto &m = *impl;
    if (!m.stop) return E2SARErrorInfo{E2SARErrorc::LogicError, "This method should only be called after the threads have been stopped."};
    std::list<std::pair<uint16_t, size_t>> out;
    for (auto &kv : m.perPort) out.emplace_back(kv.first, kv.second->load());
    return out;
}

size_t Reassembler::get_numRecvThreads() const noexcept { return impl->numRecvThreads; }
const std::pair<int, int> Reassembler::get_recvPorts() const noexcept
{
    return std::make_pair((int)impl->dataPort, (int)(impl->dataPort + impl->numRecvPorts - 1));
}
int Reassembler::get_portRange() const noexcept { return impl->portRange; }
const std::string Reassembler::get_dataIP() const noexcept { return impl->dataIP; }

const Reassembler::DeviceStats Reassembler::getDeviceStats() const noexcept
{
    auto &m = *impl;
    e2sar_hip_reas_stats st{};
    if (!m.started || e2sar_hip_reas_get_stats(m.reas, &st) != 0) {
        std::lock_guard<std::mutex> lk(m.sMu);
        st = m.lastStats;
    }
    return DeviceStats{st.tableUsed, st.arenaUsed, m.upkeeps.load(), st.inProgress, st.errorFlags};
}

void Reassembler::stopThreads()
{
    auto &m = *impl;
    if (m.stop && !m.started) return;
    m.stop = true;
    m.eCv.notify_all();
    m.bFreeCv.notify_all();
    for (auto &t : m.recvThreads)
        if (t.joinable()) t.join();
    m.bFullCv.notify_all();
    if (m.devThread.joinable()) m.devThread.join();
    m.started = false;
}

}  // namespace e2sar
