// reassembler.cpp -- e2sar::Reassembler over the gfx950 reassembly kernel.
//
// Reference: N receive threads, each owning a set of UDP ports, run the per-datagram body
// (e2sarDPReassembler.cpp:293-433) -- malloc, recvfrom, header checks, map lookup, memcpy
// -- one datagram at a time; a GC thread drops stale events (cpp:236-291).
// Here the receive threads only fill pinned datagram batches with recvmmsg (a slot of
// recvStride bytes per datagram); one device thread moves each full (or timed-out)
// batch to HBM and runs reas_kernel on it, then drains completed events (device ->
// new[] host buffers -> the event queue that getEvent/recvEvent read) and lost-event
// records, runs the device GC pass every eventTimeout_ms, and compacts the device arena
// when it fills.  Event bytes are copied to the caller's new[] buffer exactly once.
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

    // device
    e2sar_hip_ctx *ctx = nullptr;
    void *stream = nullptr;
    e2sar_hip_reas *reas = nullptr;
    uint8_t *dPkts = nullptr;
    uint32_t *dLens = nullptr;
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

    // event queue (QSIZE 1000, hpp:126) and lost events (hpp:102-122, 262-279)
    struct Ev {
        uint8_t *event;
        size_t bytes;
        EventNum_t eventNum;
        uint16_t dataId;
    };
    static constexpr size_t kQSize = 1000;
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
    void drain(bool all);
    Batch *takeFree();
};

Reassembler::Impl::~Impl()
{
    if (ctx) e2sar_hip_stream_sync(ctx, stream);
    for (auto &b : batches) {
        if (b.pkts) e2sar_hip_host_free(b.pkts);
        if (b.lens) e2sar_hip_host_free(b.lens);
    }
    if (reas) e2sar_hip_reas_destroy(reas);
    if (ctx) {
        if (dPkts) e2sar_hip_device_free(ctx, dPkts);
        if (dLens) e2sar_hip_device_free(ctx, dLens);
        e2sar_hip_ctx_destroy(ctx);
    }
    if (stream) e2sar_hip_stream_destroy(stream);
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
    if (rc == 0) rc = e2sar_hip_ctx_create(flags.gpuDevice, stream, &ctx);
    e2sar_hip_reas_config cfg{};
    cfg.withLBHeader = flags.withLBHeader ? 1 : 0;
    cfg.tableSlots = flags.tableSlots;
    cfg.queueCapacity = (uint32_t)std::max<size_t>(4096, flags.recvBatch);
    cfg.lostCapacity = 4096;
    cfg.arenaBytes = flags.arenaBytes;
    cfg.flags = E2SAR_HIP_REAS_COMPACTABLE;
    if (rc == 0) rc = e2sar_hip_reas_create(ctx, &cfg, &reas);
    if (rc == 0) rc = e2sar_hip_device_alloc(ctx, flags.recvBatch * flags.recvStride, reinterpret_cast<void **>(&dPkts));
    if (rc == 0) rc = e2sar_hip_device_alloc(ctx, flags.recvBatch * 4, reinterpret_cast<void **>(&dLens));
    const size_t nb = 2 * numRecvThreads + 2;
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
    Batch *b = takeFree();
    uint64_t firstUs = 0;
    auto flush = [&]() {
        if (!b || b->n == 0) return;
        {
            std::lock_guard<std::mutex> lk(bMu);
            fullB.push_back(b);
        }
        bFullCv.notify_one();
        b = takeFree();
        firstUs = 0;
    };
    while (!stop) {
        if (!b) {
            b = takeFree();
            if (!b) continue;
        }
        const int timeout = (b->n > 0) ? std::max(1, flags.batchTimeout_us / 1000) : 10;   // 10 ms like sleep_tv
        const int pr = poll(pf.data(), pf.size(), timeout);
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
                for (size_t k = 0; k < room; k++) {
                    iv[k].iov_base = b->pkts + (b->n + k) * S;
                    iv[k].iov_len = S;
                    mv[k].msg_hdr = msghdr{};
                    mv[k].msg_hdr.msg_iov = &iv[k];
                    mv[k].msg_hdr.msg_iovlen = 1;
                }
                const int r = recvmmsg(fds[i], mv.data(), (unsigned)room, MSG_DONTWAIT, nullptr);
                if (r < 0) {
                    if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
                        dataErrCnt++;
                        lastErrno = errno;
                    }
                    break;
                }
                for (int k = 0; k < r; k++) {
                    uint32_t len = mv[k].msg_len;
                    if (mv[k].msg_hdr.msg_flags & MSG_TRUNC) len = (uint32_t)S + 1;   // device: dataErrCnt
                    b->lens[b->n + k] = len;
                }
                perPort[ports[i]]->fetch_add((size_t)r);
                if (b->n == 0 && r > 0) firstUs = detail::now_us();
                b->n += (uint32_t)r;
                if (b->n == cap) flush();
                if (r < (int)room) break;
            }
        }
        if (b && b->n > 0 && detail::now_us() - firstUs >= (uint64_t)flags.batchTimeout_us) flush();
    }
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

// Drain completed events (device records -> new[] buffers -> event queue) and lost records.
void Reassembler::Impl::drain(bool)
{
    uint32_t n = 0;
    if (e2sar_hip_reas_poll(reas, recs.data(), (uint32_t)recs.size(), &n) != 0) {
        lastErr = E2SARErrorc::SystemError;
        return;
    }
    uint8_t *arena = e2sar_hip_reas_arena(reas);
    std::vector<Ev> ready;
    ready.reserve(n);
    for (uint32_t i = 0; i < n; i++) {
        const auto &r = recs[i];
        auto *buf = new uint8_t[r.bytes ? r.bytes : 1];
        if (r.bytes) e2sar_hip_memcpy_async(ctx, buf, arena + r.arenaOffset, r.bytes, 1, nullptr);
        ready.push_back(Ev{buf, r.bytes, r.eventNum, r.dataId});
    }
    if (n) e2sar_hip_stream_sync(ctx, nullptr);
    {
        std::lock_guard<std::mutex> lk(eMu);
        for (auto &e : ready) {
            if (evq.size() >= kQSize) {                  // enqueue loss (hpp:140-145, cpp:413-421)
                hostEnqueueLoss++;
                std::lock_guard<std::mutex> l2(lMu);
                if (lostSeen.insert({e.eventNum, e.dataId}).second) lostq.emplace_back(e.eventNum, e.dataId, 0);
                delete[] e.event;
            } else {
                evq.push_back(e);
            }
        }
    }
    if (n) eCv.notify_all();
    uint32_t nl = 0;
    if (e2sar_hip_reas_lost_poll(reas, lrecs.data(), (uint32_t)lrecs.size(), &nl) == 0 && nl) {
        std::lock_guard<std::mutex> l2(lMu);
        for (uint32_t i = 0; i < nl; i++) {   // logLostEvent dedupe (hpp:266-269)
            const auto &l = lrecs[i];
            if (lostSeen.insert({l.eventNum, l.dataId}).second) lostq.emplace_back(l.eventNum, l.dataId, l.numFragments);
        }
    }
}

void Reassembler::Impl::devBody()
{
    uint64_t lastGc = detail::steady_ms();
    while (true) {
        Batch *b = nullptr;
        {
            std::unique_lock<std::mutex> lk(bMu);
            bFullCv.wait_for(lk, std::chrono::milliseconds(10), [&] { return stop.load() || !fullB.empty(); });
            if (!fullB.empty()) {
                b = fullB.front();
                fullB.pop_front();
            } else if (stop && recvActive.load() == 0) {
                break;
            }
        }
        if (b) {
            const uint64_t now = detail::steady_ms();
            int rc = e2sar_hip_memcpy_async(ctx, dPkts, b->pkts, (size_t)b->n * flags.recvStride, 0, nullptr);
            if (rc == 0) rc = e2sar_hip_memcpy_async(ctx, dLens, b->lens, (size_t)b->n * 4, 0, nullptr);
            if (rc == 0) rc = e2sar_hip_reassemble_batch(reas, dPkts, (uint32_t)flags.recvStride, dLens, b->n, now, nullptr);
            if (rc == 0) rc = e2sar_hip_stream_sync(ctx, nullptr);
            if (rc) lastErr = static_cast<E2SARErrorc>(-rc);
            {
                std::lock_guard<std::mutex> lk(bMu);
                freeB.push_back(b);
            }
            bFreeCv.notify_all();
            drain(false);
        }
        const uint64_t now = detail::steady_ms();
        if (now - lastGc >= (uint64_t)flags.eventTimeout_ms) {    // GC thread period (cpp:252-283)
            e2sar_hip_reas_gc(reas, now, (uint64_t)flags.eventTimeout_ms, nullptr);
            lastGc = now;
            drain(false);
        }
        e2sar_hip_reas_stats st{};
        if (e2sar_hip_reas_get_stats(reas, &st) == 0) {
            {
                std::lock_guard<std::mutex> lk(sMu);
                lastStats = st;
            }
            // recycle or compact the arena once half of it is used (no completed record pending)
            if (st.completedPending == 0 && st.arenaUsed > flags.arenaBytes / 2) {
                if (st.inProgress == 0) e2sar_hip_reas_recycle(reas, 0, nullptr);
                else e2sar_hip_reas_compact(reas, nullptr);
            } else if (st.completedPending == 0 && st.inProgress == 0 && st.tableUsed > flags.tableSlots / 2) {
                e2sar_hip_reas_recycle(reas, 0, nullptr);
            }
        }
    }
    drain(true);
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
