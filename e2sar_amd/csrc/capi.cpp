// capi.cpp -- the extern "C" boundary declared in include/e2sar_hip.h.
//
// Host-side glue only: argument checks (mirroring the reference's sanity checks),
// device allocation of the reassembly state, and the hand-off of device records to
// the caller.  Every byte of event or datagram data is moved by the kernels in
// sar_kernels.hip; there is no CPU fallback.
#ifndef E2SAR_HIP_EXPERIMENTAL
#define E2SAR_HIP_EXPERIMENTAL 0
#endif
#if E2SAR_HIP_EXPERIMENTAL
#include "e2sar_hip_experimental.h"
#endif
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <set>
#include <mutex>
#include <string>
#include <vector>

#include "e2sar_hip.h"
#include "sar_kernels.hpp"

using namespace e2sar_amd;

namespace {

thread_local std::string g_lastError;

int fail(int code, const std::string &msg)
{
    g_lastError = msg;
    return code;
}

int hip_fail(hipError_t e, const char *what)
{
    return fail(E2SAR_HIP_ERR_SYSTEM, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t _e = (expr);                         \
        if (_e != hipSuccess) return hip_fail(_e, #expr); \
    } while (0)

}  // namespace

// A context is shared: every reassembler created on it holds a reference, so the caller may
// destroy the context and its reassemblers in any order (a garbage collector tearing down a
// reference cycle picks one) -- the memory goes with the last reference.
struct e2sar_hip_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::atomic<int> refs{1};
};
static void ctx_release(e2sar_hip_ctx *c)
{
    if (c && c->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) delete c;
}

struct e2sar_hip_reas {
    e2sar_hip_ctx *ctx = nullptr;
    e2sar_hip_reas_config cfg{};
    ReasDev dev{};
    ReasDev alt{};                   // second slots + arena (COMPACTABLE), same ctl/lists
    void *stateMem = nullptr;        // slots | ctl | shards | occupancy shards | completed | lost
    void *altSlots = nullptr;
    // Internal buffers, one set PER STREAM (two batches launched on different streams must
    // not share work records or ready counters while both run): the reference-order sort
    // keys / records / sort storage, the PktInfo/FinishRec work buffer of reassemble_batch
    // (reference order, or batches above kFusedMaxBytes), the chained form's ready counters.
    // They grow on demand, never inside a graph capture, and a buffer they outgrow is kept
    // (retired) until the reassembler is destroyed: a graph captured before the growth still
    // holds its address.
    struct Scratch {
        void *roScratch = nullptr;
        size_t roScratchBytes = 0;
        // a reference-order launch sequence failed part way: the key pass may have left run
        // counts that only the place / walk kernels reset, so the next batch re-zeroes them
        bool roDirty = false;
        void *roWork = nullptr;
        size_t roWorkBytes = 0;
        void *tiles = nullptr;
        size_t tilesBytes = 0;
    };
    std::map<hipStream_t, Scratch> scratch;
    std::vector<void *> retired;
    // the streams launched on outside capture: poll / lost_poll / get_stats wait for those
    // streams only, not for the whole device (an event recorded on each at snapshot time --
    // not after every launch: a marker between kernels lengthens the next kernel's start)
    std::set<hipStream_t> streams;
    hipEvent_t waitEv = nullptr;
    bool sawCapture = false;         // a launch was captured into a graph: snapshots wait for the device
    std::mutex mu;
};

static bool ref_order(const e2sar_hip_reas *r) { return (r->cfg.flags & E2SAR_HIP_REAS_REFERENCE_ORDER) != 0; }

static bool capturing(hipStream_t s)
{
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// After a launch through this reassembler on stream s (caller holds r->mu): remember the
// stream, so a later snapshot waits for exactly the streams this reassembler used.
static hipError_t note_launch(e2sar_hip_reas *r, hipStream_t s)
{
    if (capturing(s)) r->sawCapture = true;          // replays run wherever the caller puts them
    else r->streams.insert(s);
    return hipSuccess;
}

// reassemble_batch keeps the fused kernel up to this many bytes of datagram slots (a batch
// that can still sit in the 256 MiB Infinity Cache) and switches to the split form above
static constexpr uint64_t kFusedMaxBytes = 320ull << 20;

// Streaming (non-temporal) datagram loads in the scatter: for datagrams the caller declares
// cold (E2SAR_HIP_REAS_COLD_DATAGRAMS), and for a batch too large to still be cached.
static bool cold_loads(const e2sar_hip_reas *r, uint32_t n, uint32_t stride)
{
    return (r->cfg.flags & E2SAR_HIP_REAS_COLD_DATAGRAMS) != 0 || (uint64_t)n * stride > kFusedMaxBytes;
}

// Grow an internal buffer of stream s to at least `need` bytes (a quarter more, to
// amortise); caller holds r->mu.  The old buffer is retired, not freed: kernels of earlier
// batches may still read it, and a graph captured earlier holds its address.  Inside a
// capture a buffer cannot grow (allocation there would break the capture): the call fails
// with a LogicError naming the remedy instead.
static int grow(e2sar_hip_reas *r, hipStream_t s, void *&buf, size_t &have, size_t need, bool *grew = nullptr)
{
    if (grew) *grew = false;
    if (need <= have) return E2SAR_HIP_OK;
    if (capturing(s))
        return fail(E2SAR_HIP_ERR_LOGIC, "an internal buffer must grow for this batch size inside a graph capture: "
                                         "run one batch of the largest size on this stream before capturing");
    const size_t want = need + need / 4;
    void *nb = nullptr;
    hipError_t e = hipMalloc(&nb, want);
    if (e != hipSuccess) return fail(E2SAR_HIP_ERR_MEMORY, std::string("hipMalloc(internal buffer): ") + hipGetErrorString(e));
    if (buf) r->retired.push_back(buf);
    buf = nb;
    have = want;
    if (grew) *grew = true;
    return E2SAR_HIP_OK;
}

static void free_internal(e2sar_hip_reas *r)
{
    for (auto &kv : r->scratch) {
        if (kv.second.roScratch) (void)hipFree(kv.second.roScratch);
        if (kv.second.roWork) (void)hipFree(kv.second.roWork);
        if (kv.second.tiles) (void)hipFree(kv.second.tiles);
    }
    r->scratch.clear();
    for (void *p : r->retired) (void)hipFree(p);
    r->retired.clear();
    if (r->waitEv) (void)hipEventDestroy(r->waitEv);
    r->waitEv = nullptr;
    r->streams.clear();
}

// Free the internal buffers of stream s (caller holds r->mu and knows none of its launches
// still runs).  Buffers a graph capture may hold are retired instead, as in grow().
static void drop_scratch(e2sar_hip_reas *r, hipStream_t s)
{
    auto it = r->scratch.find(s);
    if (it == r->scratch.end()) return;
    for (void *p : {it->second.roScratch, it->second.roWork, it->second.tiles}) {
        if (!p) continue;
        if (r->sawCapture) r->retired.push_back(p);
        else (void)hipFree(p);
    }
    r->scratch.erase(it);
}

// Free whatever a partly built reassembler holds (every pointer starts null).
static void reas_release(e2sar_hip_reas *r)
{
    free_internal(r);
    if (r->altSlots) (void)hipFree(r->altSlots);
    if (r->alt.arena && r->alt.arena != r->dev.arena) (void)hipFree(r->alt.arena);
    if (r->dev.arena) (void)hipFree(r->dev.arena);
    if (r->stateMem) (void)hipFree(r->stateMem);
    delete r;
}

extern "C" {

int e2sar_hip_abi_version(void) { return E2SAR_HIP_ABI_VERSION; }

const char *e2sar_hip_last_error(void) { return g_lastError.c_str(); }

int e2sar_hip_ctx_create(int device, void *stream, e2sar_hip_ctx **out)
{
    if (!out) return fail(E2SAR_HIP_ERR_PARAMETER, "out is NULL");
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(E2SAR_HIP_ERR_PARAMETER, "no such device");
    HIP_TRY(hipSetDevice(device));
    auto *c = new e2sar_hip_ctx;
    c->device = device;
    c->stream = static_cast<hipStream_t>(stream);   // NULL = the device's default stream
    *out = c;
    return E2SAR_HIP_OK;
}

void e2sar_hip_ctx_destroy(e2sar_hip_ctx *ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    ctx_release(ctx);
}

int e2sar_hip_stream_create(int device, void **out)
{
    if (!out) return fail(E2SAR_HIP_ERR_PARAMETER, "out is NULL");
    HIP_TRY(hipSetDevice(device));
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *out = s;
    return E2SAR_HIP_OK;
}

int e2sar_hip_stream_destroy(void *stream)
{
    if (!stream) return E2SAR_HIP_OK;
    HIP_TRY(hipStreamDestroy(static_cast<hipStream_t>(stream)));
    return E2SAR_HIP_OK;
}

void *e2sar_hip_ctx_stream(e2sar_hip_ctx *ctx) { return ctx ? ctx->stream : nullptr; }
int e2sar_hip_ctx_device(e2sar_hip_ctx *ctx) { return ctx ? ctx->device : -1; }

int e2sar_hip_ctx_sync(e2sar_hip_ctx *ctx)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return E2SAR_HIP_OK;
}

// Large device buffers (arena, e2sar_hip_device_alloc).  (Round 3: physically contiguous
// allocations, hipDeviceMallocContiguous, made config 3's scatter 27 % slower at every
// offset)
static hipError_t dev_malloc(void **p, size_t bytes) { return hipMalloc(p, bytes); }

int e2sar_hip_device_alloc(e2sar_hip_ctx *ctx, size_t bytes, void **out)
{
    if (!ctx || !out) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL argument");
    HIP_TRY(hipSetDevice(ctx->device));
    hipError_t e = dev_malloc(out, bytes ? bytes : 1);
    if (e != hipSuccess) return fail(E2SAR_HIP_ERR_MEMORY, std::string("hipMalloc: ") + hipGetErrorString(e));
    return E2SAR_HIP_OK;
}

int e2sar_hip_device_free(e2sar_hip_ctx *ctx, void *p)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipFree(p));
    return E2SAR_HIP_OK;
}

int e2sar_hip_host_alloc(size_t bytes, void **out)
{
    if (!out) return fail(E2SAR_HIP_ERR_PARAMETER, "out is NULL");
    hipError_t e = hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault);
    if (e != hipSuccess) return fail(E2SAR_HIP_ERR_MEMORY, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    return E2SAR_HIP_OK;
}

int e2sar_hip_host_free(void *p)
{
    HIP_TRY(hipHostFree(p));
    return E2SAR_HIP_OK;
}

int e2sar_hip_memcpy_h2d(e2sar_hip_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return E2SAR_HIP_OK;
}

int e2sar_hip_memcpy_d2h(e2sar_hip_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return E2SAR_HIP_OK;
}

int e2sar_hip_memset_d(e2sar_hip_ctx *ctx, void *dst, int value, size_t bytes)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    HIP_TRY(hipSetDevice(ctx->device));
    // a fill kernel, not hipMemsetAsync: the call may be captured into a HIP graph, where
    // memset nodes misbehave on replay
    HIP_TRY(launch_fill_bytes(dst, value, bytes, ctx->stream));
    return E2SAR_HIP_OK;
}

int e2sar_hip_memset_async(e2sar_hip_ctx *ctx, void *dst, int value, size_t bytes, void *stream)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(launch_fill_bytes(dst, value, bytes, stream ? static_cast<hipStream_t>(stream) : ctx->stream));
    return E2SAR_HIP_OK;
}

int e2sar_hip_memcpy_async(e2sar_hip_ctx *ctx, void *dst, const void *src, size_t bytes, int kind, void *stream)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    if (kind < 0 || kind > 2) return fail(E2SAR_HIP_ERR_PARAMETER, "kind must be 0 (H2D), 1 (D2H) or 2 (D2D)");
    if (bytes == 0) return E2SAR_HIP_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, k, s));
    return E2SAR_HIP_OK;
}

int e2sar_hip_stream_sync(e2sar_hip_ctx *ctx, void *stream)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipStreamSynchronize(stream ? static_cast<hipStream_t>(stream) : ctx->stream));
    return E2SAR_HIP_OK;
}

int e2sar_hip_event_create(e2sar_hip_ctx *ctx, void **out)
{
    if (!ctx || !out) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL argument");
    HIP_TRY(hipSetDevice(ctx->device));
    hipEvent_t e = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    *out = e;
    return E2SAR_HIP_OK;
}

int e2sar_hip_event_destroy(void *event)
{
    if (event) HIP_TRY(hipEventDestroy(static_cast<hipEvent_t>(event)));
    return E2SAR_HIP_OK;
}

int e2sar_hip_event_record(e2sar_hip_ctx *ctx, void *event, void *stream)
{
    if (!ctx || !event) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL argument");
    HIP_TRY(hipEventRecord(static_cast<hipEvent_t>(event), stream ? static_cast<hipStream_t>(stream) : ctx->stream));
    return E2SAR_HIP_OK;
}

int e2sar_hip_stream_wait_event(e2sar_hip_ctx *ctx, void *stream, void *event)
{
    if (!ctx || !event) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL argument");
    HIP_TRY(hipStreamWaitEvent(stream ? static_cast<hipStream_t>(stream) : ctx->stream, static_cast<hipEvent_t>(event), 0));
    return E2SAR_HIP_OK;
}

int e2sar_hip_event_query(void *event)
{
    if (!event) return fail(E2SAR_HIP_ERR_PARAMETER, "event is NULL");
    const hipError_t e = hipEventQuery(static_cast<hipEvent_t>(event));
    if (e == hipSuccess) return 1;
    if (e == hipErrorNotReady) return 0;
    return hip_fail(e, "hipEventQuery");
}

int e2sar_hip_event_sync(void *event)
{
    if (!event) return fail(E2SAR_HIP_ERR_PARAMETER, "event is NULL");
    HIP_TRY(hipEventSynchronize(static_cast<hipEvent_t>(event)));
    return E2SAR_HIP_OK;
}

int e2sar_hip_copy_spans(e2sar_hip_ctx *ctx, const e2sar_hip_copy_span *spans, uint32_t n, void *stream)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    if (n == 0) return E2SAR_HIP_OK;
    if (!spans) return fail(E2SAR_HIP_ERR_PARAMETER, "spans is NULL");
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    for (uint32_t i0 = 0; i0 < n; i0 += kCopySpansPerLaunch) {
        CopySpans cs{};
        cs.n = std::min<uint32_t>(kCopySpansPerLaunch, n - i0);
        uint64_t most = 0;
        for (uint32_t k = 0; k < cs.n; k++) {
            const auto &sp = spans[i0 + k];
            if (sp.bytes && (!sp.src || !sp.dst)) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL span pointer");
            cs.s[k] = CopySpan{reinterpret_cast<uint64_t>(sp.src), reinterpret_cast<uint64_t>(sp.dst), sp.bytes};
            most = std::max<uint64_t>(most, sp.bytes);
        }
        hipError_t e = launch_copy_spans(cs, most, s);
        if (e != hipSuccess) return hip_fail(e, "copy_spans launch");
    }
    return E2SAR_HIP_OK;
}

/* ---------------- geometry ---------------- */

size_t e2sar_hip_total_hdr_len(int useIPv6)
{
    return (useIPv6 ? 40u : 20u) + 8u + E2SAR_HIP_LB_HDR_LEN + E2SAR_HIP_RE_HDR_LEN;
}

size_t e2sar_hip_max_pld_len(uint32_t mtu, int useIPv6)
{
    const size_t h = e2sar_hip_total_hdr_len(useIPv6);
    return mtu > h ? mtu - h : 0;
}

size_t e2sar_hip_num_packets(size_t bytes, size_t maxPldLen)
{
    return maxPldLen ? (bytes + maxPldLen - 1) / maxPldLen : 0;
}

uint32_t e2sar_hip_packet_stride(size_t maxPldLen)
{
    return (uint32_t)((E2SAR_HIP_LBRE_HDR_LEN + maxPldLen + 15) & ~(size_t)15);
}

/* ---------------- segmentation ---------------- */

int e2sar_hip_seg_plan(e2sar_hip_seg_event *events, uint32_t nEvents, size_t maxPldLen,
                       uint32_t *totalPackets, uint32_t *maxPacketsPerEvent)
{
    if (!events && nEvents) return fail(E2SAR_HIP_ERR_PARAMETER, "events is NULL");
    if (maxPldLen == 0) return fail(E2SAR_HIP_ERR_PARAMETER, "maxPldLen is 0 (MTU too small)");
    uint64_t total = 0;
    uint32_t mx = 0;
    for (uint32_t i = 0; i < nEvents; i++) {
        const uint64_t n = e2sar_hip_num_packets(events[i].bytes, maxPldLen);
        events[i].pktBase = (uint32_t)total;
        total += n;
        mx = std::max<uint32_t>(mx, (uint32_t)n);
        if (total > 0xFFFFFFFFull) return fail(E2SAR_HIP_ERR_OUT_OF_RANGE, "batch exceeds 2^32 packets");
    }
    if (totalPackets) *totalPackets = (uint32_t)total;
    if (maxPacketsPerEvent) *maxPacketsPerEvent = mx;
    return E2SAR_HIP_OK;
}

int e2sar_hip_segment_batch(e2sar_hip_ctx *ctx, const e2sar_hip_seg_event *d_events,
                            uint32_t nEvents, uint32_t maxPacketsPerEvent, int lbHdrVersion,
                            uint32_t maxPldLen, int eventsDwordAligned, uint8_t *d_packets,
                            uint32_t stride, uint32_t *d_lens, void *stream)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    if (nEvents == 0) return E2SAR_HIP_OK;
    if (!d_events || !d_packets) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer");
    if (maxPldLen == 0) return fail(E2SAR_HIP_ERR_PARAMETER, "maxPldLen is 0 (MTU too small)");
    if (maxPldLen > 65535u) return fail(E2SAR_HIP_ERR_PARAMETER, "maxPldLen above a UDP datagram");
    if ((stride & 15u) || stride < E2SAR_HIP_LBRE_HDR_LEN + maxPldLen)
        return fail(E2SAR_HIP_ERR_PARAMETER, "stride must be a multiple of 16 and hold 36 + maxPldLen");
    if (((uintptr_t)d_packets & 15u) != 0) return fail(E2SAR_HIP_ERR_PARAMETER, "packet buffer not 16-byte aligned");
    (void)eventsDwordAligned;        // a hint only: the kernel checks every event's address itself
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    hipError_t e = launch_segment(d_events, nEvents, maxPacketsPerEvent, lbHdrVersion, maxPldLen,
                                  d_packets, stride, d_lens, s);
    if (e != hipSuccess) return hip_fail(e, "seg_kernel launch");
    return E2SAR_HIP_OK;
}

int e2sar_hip_segment_batch_dev(e2sar_hip_ctx *ctx, const e2sar_hip_seg_event *d_events, const uint32_t *d_counts,
                                uint32_t maxEvents, uint32_t maxPacketsPerEvent, int lbHdrVersion, uint32_t maxPldLen,
                                uint8_t *d_packets, uint32_t stride, uint32_t *d_lens, void *stream)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    if (maxEvents == 0) return E2SAR_HIP_OK;
    if (!d_events || !d_counts || !d_packets) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer");
    if (maxPldLen == 0) return fail(E2SAR_HIP_ERR_PARAMETER, "maxPldLen is 0 (MTU too small)");
    if (maxPldLen > 65535u) return fail(E2SAR_HIP_ERR_PARAMETER, "maxPldLen above a UDP datagram");
    if ((stride & 15u) || stride < E2SAR_HIP_LBRE_HDR_LEN + maxPldLen)
        return fail(E2SAR_HIP_ERR_PARAMETER, "stride must be a multiple of 16 and hold 36 + maxPldLen");
    if (((uintptr_t)d_packets & 15u) != 0) return fail(E2SAR_HIP_ERR_PARAMETER, "packet buffer not 16-byte aligned");
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    hipError_t e = launch_segment(d_events, maxEvents, maxPacketsPerEvent, lbHdrVersion, maxPldLen,
                                  d_packets, stride, d_lens, s, d_counts);
    if (e != hipSuccess) return hip_fail(e, "seg_kernel launch");
    return E2SAR_HIP_OK;
}

/* ---------------- reassembly ---------------- */

int e2sar_hip_reas_create(e2sar_hip_ctx *ctx, const e2sar_hip_reas_config *cfg, e2sar_hip_reas **out)
{
    if (!ctx || !cfg || !out) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL argument");
    const uint32_t T = cfg->tableSlots;
    if (T < 64 || (T & (T - 1))) return fail(E2SAR_HIP_ERR_PARAMETER, "tableSlots must be a power of two >= 64");
    if (cfg->queueCapacity == 0 || cfg->lostCapacity == 0) return fail(E2SAR_HIP_ERR_PARAMETER, "zero capacity");
    if (cfg->groupSize > 64) return fail(E2SAR_HIP_ERR_PARAMETER, "groupSize must be 0 (auto) or 1..64");
    HIP_TRY(hipSetDevice(ctx->device));
    auto *r = new e2sar_hip_reas;
    r->ctx = ctx;
    r->cfg = *cfg;
    const size_t slotsB = sizeof(ReasSlot) * (size_t)T;
    const size_t ctlB = sizeof(ReasCtl) + (sizeof(ReasShard) + sizeof(ReasOcc)) * kShards;
    const size_t compB = sizeof(e2sar_hip_event_rec) * (size_t)cfg->queueCapacity;
    const size_t lostB = sizeof(e2sar_hip_lost_rec) * (size_t)cfg->lostCapacity;
    const size_t total = slotsB + ctlB + compB + lostB;
    hipError_t e = hipMalloc(&r->stateMem, total);
    if (e != hipSuccess) {
        r->stateMem = nullptr;
        reas_release(r);
        return fail(E2SAR_HIP_ERR_MEMORY, std::string("hipMalloc(state): ") + hipGetErrorString(e));
    }
    e = dev_malloc(reinterpret_cast<void **>(&r->dev.arena), cfg->arenaBytes ? cfg->arenaBytes : 256);
    if (e != hipSuccess) {
        r->dev.arena = nullptr;
        reas_release(r);
        return fail(E2SAR_HIP_ERR_MEMORY, std::string("hipMalloc(arena): ") + hipGetErrorString(e));
    }
    // reas_stream_kernel takes a payload's 16-byte phase in its event buffer from the
    // datagram's bufferOffset alone: event buffers are 256-byte aligned in a 256-byte-aligned arena
    if ((reinterpret_cast<uintptr_t>(r->dev.arena) & 255u) != 0) {
        reas_release(r);
        return fail(E2SAR_HIP_ERR_MEMORY, "arena not 256-byte aligned");
    }
    auto *base = static_cast<uint8_t *>(r->stateMem);
    r->dev.slots = reinterpret_cast<ReasSlot *>(base);
    r->dev.ctl = reinterpret_cast<ReasCtl *>(base + slotsB);
    r->dev.shards = reinterpret_cast<ReasShard *>(base + slotsB + sizeof(ReasCtl));
    r->dev.completed = reinterpret_cast<e2sar_hip_event_rec *>(base + slotsB + ctlB);
    r->dev.lost = reinterpret_cast<e2sar_hip_lost_rec *>(base + slotsB + ctlB + compB);
    r->dev.arenaBytes = cfg->arenaBytes;
    r->dev.tableSlots = T;
    r->dev.queueCapacity = cfg->queueCapacity;
    r->dev.lostCapacity = cfg->lostCapacity;
    r->dev.withLB = cfg->withLBHeader ? 1 : 0;
    r->dev.ownWorld = 1;                       // every event is ours until set_owner
    r->dev.ownSelf = 0;
    r->dev.groupSize = cfg->groupSize;
    r->alt = r->dev;
    r->alt.arena = nullptr;
    if (cfg->flags & E2SAR_HIP_REAS_COMPACTABLE) {
        e = hipMalloc(&r->altSlots, slotsB);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&r->alt.arena), cfg->arenaBytes ? cfg->arenaBytes : 256);
        if (e != hipSuccess) {
            reas_release(r);
            return fail(E2SAR_HIP_ERR_MEMORY, std::string("hipMalloc(alternate arena): ") + hipGetErrorString(e));
        }
        r->alt.slots = reinterpret_cast<ReasSlot *>(r->altSlots);
        e = hipMemsetAsync(r->altSlots, 0, slotsB, ctx->stream);
        if (e != hipSuccess) {
            reas_release(r);
            return hip_fail(e, "alternate table init");
        }
    } else {
        r->alt.slots = nullptr;
        r->alt.arena = nullptr;
    }
    e = hipMemsetAsync(r->stateMem, 0, total, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        reas_release(r);
        return hip_fail(e, "state init");
    }
    ctx->refs.fetch_add(1, std::memory_order_relaxed);          // released by e2sar_hip_reas_destroy
    *out = r;
    return E2SAR_HIP_OK;
}

void e2sar_hip_reas_destroy(e2sar_hip_reas *r)
{
    if (!r) return;
    (void)hipSetDevice(r->ctx->device);
    // launches on any stream (the caller's, a graph replay's) may still use the table, the
    // arena and the internal buffers: wait for the device before the first hipFree
    (void)hipDeviceSynchronize();
    if (r->alt.slots) {
        // the two tables/arenas may have been swapped: free whichever is not in stateMem
        auto *base = static_cast<uint8_t *>(r->stateMem);
        ReasSlot *inState = reinterpret_cast<ReasSlot *>(base);
        (void)hipFree(r->dev.slots == inState ? static_cast<void *>(r->alt.slots) : static_cast<void *>(r->dev.slots));
        (void)hipFree(r->alt.arena);
    }
    (void)hipFree(r->dev.arena);
    (void)hipFree(r->stateMem);
    free_internal(r);
    e2sar_hip_ctx *ctx = r->ctx;
    delete r;
    ctx_release(ctx);
}

uint8_t *e2sar_hip_reas_arena(e2sar_hip_reas *r) { return r ? r->dev.arena : nullptr; }

}  // extern "C"

// Scratch of the reference-order classification for n datagrams on stream s (caller holds r->mu).
static int ro_prepare(e2sar_hip_reas *r, hipStream_t s, uint32_t n)
{
    // the run counters at the front are zero between batches (the kernels reset what they
    // use); a new buffer starts them at zero
    auto &sc = r->scratch[s];
    bool grew = false;
    if (int rc = grow(r, s, sc.roScratch, sc.roScratchBytes, ro_scratch_bytes(n, r->dev.tableSlots), &grew)) return rc;
    if (grew) HIP_TRY(hipMemsetAsync(sc.roScratch, 0, ro_zero_bytes(r->dev.tableSlots), s));
    else if (sc.roDirty) HIP_TRY(launch_fill_bytes(sc.roScratch, 0, ro_zero_bytes(r->dev.tableSlots), s));  // capture-safe
    sc.roDirty = false;
    return E2SAR_HIP_OK;
}

// launch_ro_classify, remembering a failure part way through its launches (ro_prepare)
static hipError_t ro_classify(e2sar_hip_reas *r, hipStream_t s, const uint8_t *pk, uint32_t stride, const uint32_t *lens,
                              uint32_t n, uint64_t now, void *work)
{
    auto &sc = r->scratch[s];
    const hipError_t e = launch_ro_classify(r->dev, pk, stride, lens, n, now, work, sc.roScratch, sc.roScratchBytes, s);
    if (e != hipSuccess) sc.roDirty = true;
    return e;
}

extern "C" {

int e2sar_hip_reassemble_batch(e2sar_hip_reas *r, const uint8_t *d_packets, uint32_t stride,
                               const uint32_t *d_lens, uint32_t nPackets, uint64_t now_ms, void *stream)
{
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    if (nPackets == 0) return E2SAR_HIP_OK;
    if (!d_packets || !d_lens) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer");
    const uint32_t hl = r->cfg.withLBHeader ? E2SAR_HIP_LBRE_HDR_LEN : E2SAR_HIP_RE_HDR_LEN;
    if ((stride & 15u) || stride < hl + 16u) return fail(E2SAR_HIP_ERR_PARAMETER, "stride must be a multiple of 16 and > header + 16");
    if (((uintptr_t)d_packets & 15u) != 0) return fail(E2SAR_HIP_ERR_PARAMETER, "packet buffer not 16-byte aligned");
    if ((uint64_t)nPackets * (stride >> 4) > 0xFFFFFFFFull) return fail(E2SAR_HIP_ERR_OUT_OF_RANGE, "batch too large");
    std::lock_guard<std::mutex> lk(r->mu);
    HIP_TRY(hipSetDevice(r->ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->ctx->stream;
    auto &sc = r->scratch[s];
    if (ref_order(r)) {
        // classify in arrival order into the internal work buffer, then the scatter kernel
        if (int rc = ro_prepare(r, s, nPackets)) return rc;
        if (int rc = grow(r, s, sc.roWork, sc.roWorkBytes, work_bytes(nPackets))) return rc;
        hipError_t e = ro_classify(r, s, d_packets, stride, d_lens, nPackets, now_ms, sc.roWork);
        if (e == hipSuccess)
            e = launch_reas_scatter(r->dev, d_packets, stride, nPackets, sc.roWork, s, cold_loads(r, nPackets, stride));
        if (e == hipSuccess) e = note_launch(r, s);
        if (e != hipSuccess) return hip_fail(e, "reference-order reassembly launch");
        return E2SAR_HIP_OK;
    }
    // A batch whose datagrams cannot still be in the 256 MiB Infinity Cache (more than
    // kFusedMaxBytes of slots) is read back from HBM whatever the caller did before, and
    // there the split form -- classify, then one-round scatter workgroups with streaming
    // loads -- is the faster one: 8 MiB events at MTU 9000, 70 per launch (65,730
    // datagrams, BASELINE config 3): 1116 GiB/s fused vs 1302 split.  Internal work buffer
    // of this stream, grown on first use (outside graph capture).
    if ((uint64_t)nPackets * stride > kFusedMaxBytes) {
        if (int rc = grow(r, s, sc.roWork, sc.roWorkBytes, work_bytes(nPackets))) return rc;
        hipError_t e = launch_reas_classify(r->dev, d_packets, stride, d_lens, nPackets, now_ms, sc.roWork, s);
        if (e == hipSuccess) e = launch_reas_scatter(r->dev, d_packets, stride, nPackets, sc.roWork, s, true);
        if (e == hipSuccess) e = note_launch(r, s);
        if (e != hipSuccess) return hip_fail(e, "reassembly launch (split form)");
        return E2SAR_HIP_OK;
    }
    hipError_t e = launch_reassemble(r->dev, d_packets, stride, d_lens, nPackets, now_ms, s);
    if (e == hipSuccess) e = note_launch(r, s);
    if (e != hipSuccess) return hip_fail(e, "reassembly launch");
    return E2SAR_HIP_OK;
}

#if E2SAR_HIP_EXPERIMENTAL
int e2sar_hip_seg_groups(const e2sar_hip_seg_event *events, uint32_t nEvents, uint32_t maxPacketsPerEvent,
                         uint32_t maxPldLen, uint32_t stride, uint32_t *starts, uint32_t cap, uint32_t *nGroups)
{
    if (!nGroups) return fail(E2SAR_HIP_ERR_PARAMETER, "nGroups is NULL");
    *nGroups = 0;
    if (nEvents && (!events || !starts)) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL table");
    if (maxPldLen == 0) return fail(E2SAR_HIP_ERR_PARAMETER, "maxPldLen is 0 (MTU too small)");
    if ((stride & 15u) || stride < E2SAR_HIP_LBRE_HDR_LEN + maxPldLen)
        return fail(E2SAR_HIP_ERR_PARAMETER, "stride must be a multiple of 16 and hold 36 + maxPldLen");
    *nGroups = seg_groups(events, nEvents, maxPacketsPerEvent, maxPldLen, stride, starts, cap);
    return E2SAR_HIP_OK;
}

int e2sar_hip_reassemble_groups(e2sar_hip_reas *r, const uint8_t *d_packets, uint32_t stride,
                                const uint32_t *d_lens, uint32_t nPackets, const uint32_t *d_starts,
                                uint32_t nGroups, uint64_t now_ms, void *stream)
{
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    if (nPackets == 0) return E2SAR_HIP_OK;
    if (nGroups == 0 || !d_starts || ref_order(r) || (uint64_t)nPackets * stride > kFusedMaxBytes)
        return e2sar_hip_reassemble_batch(r, d_packets, stride, d_lens, nPackets, now_ms, stream);
    if (!d_packets || !d_lens) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer");
    const uint32_t hl = r->cfg.withLBHeader ? E2SAR_HIP_LBRE_HDR_LEN : E2SAR_HIP_RE_HDR_LEN;
    if ((stride & 15u) || stride < hl + 16u) return fail(E2SAR_HIP_ERR_PARAMETER, "stride must be a multiple of 16 and > header + 16");
    if (((uintptr_t)d_packets & 15u) != 0) return fail(E2SAR_HIP_ERR_PARAMETER, "packet buffer not 16-byte aligned");
    if ((uint64_t)nPackets * (stride >> 4) > 0xFFFFFFFFull) return fail(E2SAR_HIP_ERR_OUT_OF_RANGE, "batch too large");
    if (nGroups > 0x7FFFFFFFu) return fail(E2SAR_HIP_ERR_PARAMETER, "too many groups");
    std::lock_guard<std::mutex> lk(r->mu);
    HIP_TRY(hipSetDevice(r->ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->ctx->stream;
    hipError_t e = launch_reassemble_groups(r->dev, d_packets, stride, d_lens, nPackets, d_starts, nGroups, now_ms, s);
    if (e == hipSuccess) e = note_launch(r, s);
    if (e != hipSuccess) return hip_fail(e, "reassembly launch (groups)");
    return E2SAR_HIP_OK;
}

static int segreas(e2sar_hip_ctx *ctx, const e2sar_hip_segreas_batch *batches, uint32_t nBatches, int lbHdrVersion,
                   uint32_t maxPldLen, uint32_t stride, e2sar_hip_reas *r, uint64_t now_ms, void *stream)
{
    if (!ctx || !r || (!batches && nBatches)) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL argument");
    if (nBatches > kChainMaxBatches) return fail(E2SAR_HIP_ERR_PARAMETER, "more than 8 batches per launch");
    if (maxPldLen == 0) return fail(E2SAR_HIP_ERR_PARAMETER, "maxPldLen is 0 (MTU too small)");
    if (maxPldLen > 65535u) return fail(E2SAR_HIP_ERR_PARAMETER, "maxPldLen above a UDP datagram");
    if ((stride & 15u) || stride < E2SAR_HIP_LBRE_HDR_LEN + maxPldLen)
        return fail(E2SAR_HIP_ERR_PARAMETER, "stride must be a multiple of 16 and hold 36 + maxPldLen");
    if (!r->cfg.withLBHeader) return fail(E2SAR_HIP_ERR_PARAMETER, "the chained form emits LB headers: withLBHeader required");
    if (ref_order(r)) return fail(E2SAR_HIP_ERR_PARAMETER, "the chained form is order-insensitive (no REFERENCE_ORDER)");
    ChainBatches cb{};
    uint64_t words = 0;
    for (uint32_t b = 0; b < nBatches; b++) {
        const e2sar_hip_segreas_batch &x = batches[b];
        if (x.nEvents == 0 || x.nPackets == 0) continue;
        if (!x.d_events || !x.d_packets || !x.d_lens) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer");
        if (((uintptr_t)x.d_packets & 15u) != 0) return fail(E2SAR_HIP_ERR_PARAMETER, "packet buffer not 16-byte aligned");
        if ((uint64_t)x.nPackets * (stride >> 4) > 0xFFFFFFFFull) return fail(E2SAR_HIP_ERR_OUT_OF_RANGE, "batch too large");
        for (uint32_t c = 0; c < b; c++)
            if (batches[c].d_packets == x.d_packets && batches[c].nPackets)
                return fail(E2SAR_HIP_ERR_PARAMETER, "batches of one launch need distinct packet buffers");
        ChainBatch &B = cb.b[cb.nb++];
        B.events = x.d_events;
        B.pkts = x.d_packets;
        B.lens = x.d_lens;
        B.nEvents = x.nEvents;
        B.maxPacketsPerEvent = x.maxPacketsPerEvent;
        B.n = x.nPackets;
        B.tiles = reinterpret_cast<uint32_t *>(words);        // offset for now
        words += x.nPackets;
    }
    if (cb.nb == 0) return E2SAR_HIP_OK;
    std::lock_guard<std::mutex> lk(r->mu);
    HIP_TRY(hipSetDevice(r->ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->ctx->stream;
    auto &sc = r->scratch[s];
    if (int rc = grow(r, s, sc.tiles, sc.tilesBytes, 4ull * words)) return rc;
    for (uint32_t b = 0; b < cb.nb; b++)
        cb.b[b].tiles = static_cast<uint32_t *>(sc.tiles) + reinterpret_cast<uintptr_t>(cb.b[b].tiles);
    // the launch's ready counters start at 0: zeroed by a kernel (capture-safe)
    // before every launch, so a group that gave up waiting in an earlier launch (error bit 4)
    // cannot leave a count behind for this one
    hipError_t e = launch_zero_words(sc.tiles, words, s);
    if (e == hipSuccess) e = launch_segreas(cb, lbHdrVersion, maxPldLen, stride, r->dev, now_ms, s);
    if (e == hipSuccess) e = note_launch(r, s);
    if (e != hipSuccess) return hip_fail(e, "segreas_kernel launch");
    return E2SAR_HIP_OK;
}

int e2sar_hip_segment_reassemble_batch(e2sar_hip_ctx *ctx, const e2sar_hip_seg_event *d_events, uint32_t nEvents,
                                       uint32_t maxPacketsPerEvent, uint32_t nPackets, int lbHdrVersion,
                                       uint32_t maxPldLen, uint8_t *d_packets, uint32_t stride, uint32_t *d_lens,
                                       e2sar_hip_reas *r, uint64_t now_ms, void *stream)
{
    const e2sar_hip_segreas_batch b{d_events, d_packets, d_lens, nEvents, maxPacketsPerEvent, nPackets, 0u};
    return segreas(ctx, &b, 1u, lbHdrVersion, maxPldLen, stride, r, now_ms, stream);
}

int e2sar_hip_segment_reassemble_batches(e2sar_hip_ctx *ctx, const e2sar_hip_segreas_batch *batches,
                                         uint32_t nBatches, int lbHdrVersion, uint32_t maxPldLen, uint32_t stride,
                                         e2sar_hip_reas *r, uint64_t now_ms, void *stream)
{
    return segreas(ctx, batches, nBatches, lbHdrVersion, maxPldLen, stride, r, now_ms, stream);
}

#endif  // E2SAR_HIP_EXPERIMENTAL

int e2sar_hip_relay_plan(e2sar_hip_reas *r, uint32_t firstRecord, uint32_t maxEvents, size_t maxPldLen,
                         uint64_t lbTick, uint16_t entropyBase, e2sar_hip_seg_event *d_events, uint32_t *d_counts,
                         void *stream)
{
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    if (!d_events || !d_counts) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer");
    if (maxPldLen == 0 || maxPldLen > 65535u) return fail(E2SAR_HIP_ERR_PARAMETER, "bad maxPldLen");
    std::lock_guard<std::mutex> lk(r->mu);
    HIP_TRY(hipSetDevice(r->ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->ctx->stream;
    hipError_t e = launch_relay_plan(r->dev, firstRecord, maxEvents, (uint32_t)maxPldLen, lbTick, entropyBase,
                                     d_events, d_counts, s);
    if (e == hipSuccess) e = note_launch(r, s);
    if (e != hipSuccess) return hip_fail(e, "relay_plan launch");
    return E2SAR_HIP_OK;
}

static int check_batch(e2sar_hip_reas *r, const uint8_t *d_packets, uint32_t stride, uint32_t nPackets)
{
    const uint32_t hl = r->cfg.withLBHeader ? E2SAR_HIP_LBRE_HDR_LEN : E2SAR_HIP_RE_HDR_LEN;
    if ((stride & 15u) || stride < hl + 16u) return fail(E2SAR_HIP_ERR_PARAMETER, "stride must be a multiple of 16 and > header + 16");
    if (((uintptr_t)d_packets & 15u) != 0) return fail(E2SAR_HIP_ERR_PARAMETER, "packet buffer not 16-byte aligned");
    if ((uint64_t)nPackets * (stride >> 4) > 0xFFFFFFFFull) return fail(E2SAR_HIP_ERR_OUT_OF_RANGE, "batch too large");
    return E2SAR_HIP_OK;
}

size_t e2sar_hip_reas_work_bytes(uint32_t nPackets) { return work_bytes(nPackets); }

int e2sar_hip_reas_classify(e2sar_hip_reas *r, const uint8_t *d_packets, uint32_t stride,
                            const uint32_t *d_lens, uint32_t nPackets, uint64_t now_ms,
                            void *d_work, size_t workBytes, void *stream)
{
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    if (nPackets == 0) return E2SAR_HIP_OK;
    if (!d_packets || !d_lens || !d_work) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer");
    if (((uintptr_t)d_work & 255u) != 0) return fail(E2SAR_HIP_ERR_PARAMETER, "work buffer not 256-byte aligned");
    if (workBytes < work_bytes(nPackets)) return fail(E2SAR_HIP_ERR_PARAMETER, "work buffer too small");
    if (int st = check_batch(r, d_packets, stride, nPackets)) return st;
    std::lock_guard<std::mutex> lk(r->mu);
    HIP_TRY(hipSetDevice(r->ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->ctx->stream;
    hipError_t e;
    if (ref_order(r)) {
        if (int rc = ro_prepare(r, s, nPackets)) return rc;
        e = ro_classify(r, s, d_packets, stride, d_lens, nPackets, now_ms, d_work);
    } else {
        e = launch_reas_classify(r->dev, d_packets, stride, d_lens, nPackets, now_ms, d_work, s);
    }
    if (e == hipSuccess) e = note_launch(r, s);
    if (e != hipSuccess) return hip_fail(e, "classify launch");
    return E2SAR_HIP_OK;
}

int e2sar_hip_reas_scatter(e2sar_hip_reas *r, const uint8_t *d_packets, uint32_t stride, uint32_t nPackets,
                           const void *d_work, size_t workBytes, void *stream)
{
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    if (nPackets == 0) return E2SAR_HIP_OK;
    if (!d_packets || !d_work) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer");
    if (((uintptr_t)d_work & 255u) != 0) return fail(E2SAR_HIP_ERR_PARAMETER, "work buffer not 256-byte aligned");
    if (workBytes < work_bytes(nPackets)) return fail(E2SAR_HIP_ERR_PARAMETER, "work buffer too small");
    if (int st = check_batch(r, d_packets, stride, nPackets)) return st;
    std::lock_guard<std::mutex> lk(r->mu);
    HIP_TRY(hipSetDevice(r->ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->ctx->stream;
    hipError_t e = launch_reas_scatter(r->dev, d_packets, stride, nPackets, d_work, s, cold_loads(r, nPackets, stride));
    if (e == hipSuccess) e = note_launch(r, s);
    if (e != hipSuccess) return hip_fail(e, "scatter launch");
    return E2SAR_HIP_OK;
}

int e2sar_hip_reas_scatter_classify(e2sar_hip_reas *r, uint32_t stride, const uint8_t *d_spk, uint32_t sn,
                                    const void *d_swork, size_t sworkBytes, const uint8_t *d_cpk,
                                    const uint32_t *d_clens, uint32_t cn, uint64_t now_ms, void *d_cwork,
                                    size_t cworkBytes, void *stream)
{
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    if (sn == 0 && cn == 0) return E2SAR_HIP_OK;
    if (sn) {
        if (!d_spk || !d_swork) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer (scatter batch)");
        if (((uintptr_t)d_swork & 255u) != 0) return fail(E2SAR_HIP_ERR_PARAMETER, "work buffer not 256-byte aligned");
        if (sworkBytes < work_bytes(sn)) return fail(E2SAR_HIP_ERR_PARAMETER, "scatter work buffer too small");
        if (int st = check_batch(r, d_spk, stride, sn)) return st;
    }
    if (cn) {
        if (!d_cpk || !d_clens || !d_cwork) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer (classify batch)");
        if (((uintptr_t)d_cwork & 255u) != 0) return fail(E2SAR_HIP_ERR_PARAMETER, "work buffer not 256-byte aligned");
        if (cworkBytes < work_bytes(cn)) return fail(E2SAR_HIP_ERR_PARAMETER, "classify work buffer too small");
        if (int st = check_batch(r, d_cpk, stride, cn)) return st;
    }
    if (sn && cn && d_swork == d_cwork) return fail(E2SAR_HIP_ERR_PARAMETER, "the two batches need different work buffers");
    std::lock_guard<std::mutex> lk(r->mu);
    HIP_TRY(hipSetDevice(r->ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->ctx->stream;
    hipError_t e;
    if (ref_order(r)) {
        // arrival order needs the classification of b+1 after that of b, not inside the
        // scatter of b: two launches, same results.  (Round 5: the classification of b+1 on
        // a side stream beside the scatter of b measured slower -- the scatter 63 -> 102-113
        // us beside it, DESIGN.md 3 -- so the two run in line.)
        e = launch_reas_scatter(r->dev, d_spk, stride, sn, d_swork, s, cold_loads(r, sn, stride));
        if (e == hipSuccess && cn) {
            if (int rc = ro_prepare(r, s, cn)) return rc;
            e = ro_classify(r, s, d_cpk, stride, d_clens, cn, now_ms, d_cwork);
        }
    } else {
        e = launch_reas_scatter_classify(r->dev, stride, d_spk, sn, d_swork, d_cpk, d_clens, cn, now_ms, d_cwork, s,
                                         cold_loads(r, sn, stride));
    }
    if (e == hipSuccess) e = note_launch(r, s);
    if (e != hipSuccess) return hip_fail(e, "scatter_classify launch");
    return E2SAR_HIP_OK;
}

int e2sar_hip_reas_gc(e2sar_hip_reas *r, uint64_t now_ms, uint64_t timeout_ms, void *stream)
{
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    std::lock_guard<std::mutex> lk(r->mu);
    HIP_TRY(hipSetDevice(r->ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->ctx->stream;
    hipError_t e = launch_gc(r->dev, now_ms, timeout_ms, s);
    if (e == hipSuccess) e = note_launch(r, s);
    if (e != hipSuccess) return hip_fail(e, "gc launch");
    return E2SAR_HIP_OK;
}

// Wait until every kernel launched through this reassembler has finished (caller holds
// r->mu, so no new one starts): an event recorded now on each stream it launched on, not
// the whole device -- other reassemblers, copy streams and unrelated work run on, and a
// capture in progress on another thread is not disturbed.  A stream the caller destroyed
// since (its handle no longer valid) finished its work when it was destroyed.  Once a
// launch of this reassembler has been captured into a graph, its replays can run on any
// stream, so the wait falls back to the device.
static int wait_launches(e2sar_hip_reas *r)
{
    HIP_TRY(hipSetDevice(r->ctx->device));
    if (r->sawCapture) {
        HIP_TRY(hipDeviceSynchronize());
        return E2SAR_HIP_OK;
    }
    if (!r->waitEv) HIP_TRY(hipEventCreateWithFlags(&r->waitEv, hipEventDisableTiming));
    for (auto it = r->streams.begin(); it != r->streams.end();) {
        const hipError_t e = hipEventRecord(r->waitEv, *it);
        if (e == hipErrorInvalidHandle || e == hipErrorContextIsDestroyed || e == hipErrorInvalidResourceHandle) {
            // a stream destroyed without e2sar_hip_reas_forget_stream: its work finished when
            // it was destroyed; its scratch goes with it
            (void)hipGetLastError();
            drop_scratch(r, *it);
            it = r->streams.erase(it);
            continue;
        }
        if (e != hipSuccess) return hip_fail(e, "hipEventRecord");
        HIP_TRY(hipEventSynchronize(r->waitEv));
        ++it;
    }
    // every launch of this reassembler has finished and none was captured, so no kernel and
    // no graph can still hold a buffer that an earlier growth retired
    for (void *p : r->retired) (void)hipFree(p);
    r->retired.clear();
    return E2SAR_HIP_OK;
}

// The control block with its occupancy counters live: ReasCtl's base plus the ReasOcc shards.
static int read_ctl_occ(e2sar_hip_reas *r, ReasCtl &c)
{
    HIP_TRY(hipMemcpy(&c, r->dev.ctl, sizeof(ReasCtl), hipMemcpyDeviceToHost));
    std::vector<ReasOcc> oc(kShards);
    HIP_TRY(hipMemcpy(oc.data(), r->dev.shards + kShards, sizeof(ReasOcc) * kShards, hipMemcpyDeviceToHost));
    long long used = c.tableUsed;
    for (const auto &x : oc) {
        c.inProgress += x.inProgress;
        used += x.tableUsed;
    }
    c.tableUsed = (uint32_t)used;
    return E2SAR_HIP_OK;
}

// Snapshot of the control block after every launch of this reassembler finished
// (wait_launches), so the read-modify-write of the list counts in poll / lost_poll cannot
// race a kernel's completion atomics.  With `sum` (get_stats) the per-packet shards are
// summed into it and the occupancy counters folded into c; poll / lost_poll need only the
// list counts.
static int read_ctl(e2sar_hip_reas *r, ReasCtl &c, ReasShard *sum = nullptr)
{
    if (int rc = wait_launches(r)) return rc;
    if (!sum) {
        HIP_TRY(hipMemcpy(&c, r->dev.ctl, sizeof(ReasCtl), hipMemcpyDeviceToHost));
    } else {
        if (int rc = read_ctl_occ(r, c)) return rc;
        std::vector<ReasShard> sh(kShards);
        HIP_TRY(hipMemcpy(sh.data(), r->dev.shards, sizeof(ReasShard) * kShards, hipMemcpyDeviceToHost));
        *sum = ReasShard{};
        for (const auto &x : sh) {
            sum->totalPackets += x.totalPackets;
            sum->totalBytes += x.totalBytes;
            sum->badHeaderDiscards += x.badHeaderDiscards;
            sum->dataErrCnt += x.dataErrCnt;
            sum->eventSuccess += x.eventSuccess;
        }
    }
    return E2SAR_HIP_OK;
}

}  // extern "C"

// Keep records [n, avail) queued by moving them to the front.  hipMemcpy does not allow
// overlapping ranges, so the move goes in chunks of at most n records (each chunk's
// source starts n records above its destination: they never overlap).
template <typename Rec>
static int slide_down(Rec *base, uint32_t n, uint32_t avail)
{
    if (n == 0 || n >= avail) return E2SAR_HIP_OK;
    for (uint32_t d = 0; d < avail - n; d += n) {
        const uint32_t k = std::min(n, avail - n - d);
        HIP_TRY(hipMemcpy(base + d, base + d + n, sizeof(Rec) * k, hipMemcpyDeviceToDevice));
    }
    return E2SAR_HIP_OK;
}

extern "C" {

int e2sar_hip_reas_poll(e2sar_hip_reas *r, e2sar_hip_event_rec *out, uint32_t cap, uint32_t *nOut)
{
    if (!r || !nOut || (!out && cap)) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL argument");
    std::lock_guard<std::mutex> lk(r->mu);
    ReasCtl c;
    int rc = read_ctl(r, c);
    if (rc) return rc;
    const uint32_t avail = std::min(c.nCompleted, r->dev.queueCapacity);
    const uint32_t n = std::min(avail, cap);
    if (n) HIP_TRY(hipMemcpy(out, r->dev.completed, sizeof(e2sar_hip_event_rec) * n, hipMemcpyDeviceToHost));
    if (int rc2 = slide_down(r->dev.completed, n, avail)) return rc2;
    const uint32_t left = avail - n;
    HIP_TRY(hipMemcpy(&r->dev.ctl->nCompleted, &left, sizeof(uint32_t), hipMemcpyHostToDevice));
    *nOut = n;
    return E2SAR_HIP_OK;
}

int e2sar_hip_reas_lost_poll(e2sar_hip_reas *r, e2sar_hip_lost_rec *out, uint32_t cap, uint32_t *nOut)
{
    if (!r || !nOut || (!out && cap)) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL argument");
    std::lock_guard<std::mutex> lk(r->mu);
    ReasCtl c;
    int rc = read_ctl(r, c);
    if (rc) return rc;
    const uint32_t avail = std::min(c.nLost, r->dev.lostCapacity);
    const uint32_t n = std::min(avail, cap);
    if (n) HIP_TRY(hipMemcpy(out, r->dev.lost, sizeof(e2sar_hip_lost_rec) * n, hipMemcpyDeviceToHost));
    if (int rc2 = slide_down(r->dev.lost, n, avail)) return rc2;
    const uint32_t left = avail - n;
    HIP_TRY(hipMemcpy(&r->dev.ctl->nLost, &left, sizeof(uint32_t), hipMemcpyHostToDevice));
    *nOut = n;
    return E2SAR_HIP_OK;
}

int e2sar_hip_reas_get_stats(e2sar_hip_reas *r, e2sar_hip_reas_stats *out)
{
    if (!r || !out) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL argument");
    std::lock_guard<std::mutex> lk(r->mu);
    ReasCtl c;
    ReasShard t;
    int rc = read_ctl(r, c, &t);
    if (rc) return rc;
    out->enqueueLoss = c.enqueueLoss;
    out->reassemblyLoss = c.reassemblyLoss;
    out->eventSuccess = c.eventSuccess + t.eventSuccess;
    out->totalPackets = t.totalPackets;
    out->totalBytes = t.totalBytes;
    out->badHeaderDiscards = t.badHeaderDiscards;
    out->dataErrCnt = t.dataErrCnt;
    out->inProgress = c.inProgress;
    out->completedPending = std::min(c.nCompleted, r->dev.queueCapacity);
    out->lostPending = std::min(c.nLost, r->dev.lostCapacity);
    out->arenaUsed = c.arenaTop;
    out->tableUsed = c.tableUsed;
    out->errorFlags = c.errorFlags;
    out->reserved = 0;
    return E2SAR_HIP_OK;
}

// e2sar_hip_reas_recycle's precondition (caller holds r->mu): without force, the device
// is drained and no event is in progress or unpolled
static int recycle_check(e2sar_hip_reas *r, int force, hipStream_t s)
{
    if (force) return E2SAR_HIP_OK;
    ReasCtl c;
    if (int rc = wait_launches(r)) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    if (int rc = read_ctl_occ(r, c)) return rc;
    if (c.inProgress != 0) return fail(E2SAR_HIP_ERR_LOGIC, "events still in progress");
    if (c.nCompleted != 0) return fail(E2SAR_HIP_ERR_LOGIC, "completed events not yet polled");
    return E2SAR_HIP_OK;
}

int e2sar_hip_reas_recycle(e2sar_hip_reas *r, int force, void *stream)
{
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    std::lock_guard<std::mutex> lk(r->mu);
    HIP_TRY(hipSetDevice(r->ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->ctx->stream;
    if (int rc = recycle_check(r, force, s)) return rc;
    hipError_t e = launch_recycle(r->dev, force != 0, s);
    if (e == hipSuccess) e = note_launch(r, s);
    if (e != hipSuccess) return hip_fail(e, "recycle launch");
    return E2SAR_HIP_OK;
}

int e2sar_hip_segment_batch_recycle(e2sar_hip_ctx *ctx, const e2sar_hip_seg_event *d_events, uint32_t nEvents,
                                    uint32_t maxPacketsPerEvent, int lbHdrVersion, uint32_t maxPldLen,
                                    int eventsDwordAligned, uint8_t *d_packets, uint32_t stride, uint32_t *d_lens,
                                    e2sar_hip_reas *r, int force, void *stream)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    if (r->ctx->device != ctx->device) return fail(E2SAR_HIP_ERR_PARAMETER, "reassembler on another device");
    if (nEvents && (!d_events || !d_packets)) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer");
    if (maxPldLen == 0) return fail(E2SAR_HIP_ERR_PARAMETER, "maxPldLen is 0 (MTU too small)");
    if (maxPldLen > 65535u) return fail(E2SAR_HIP_ERR_PARAMETER, "maxPldLen above a UDP datagram");
    if ((stride & 15u) || stride < E2SAR_HIP_LBRE_HDR_LEN + maxPldLen)
        return fail(E2SAR_HIP_ERR_PARAMETER, "stride must be a multiple of 16 and hold 36 + maxPldLen");
    if (((uintptr_t)d_packets & 15u) != 0) return fail(E2SAR_HIP_ERR_PARAMETER, "packet buffer not 16-byte aligned");
    (void)eventsDwordAligned;
    std::lock_guard<std::mutex> lk(r->mu);
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    if (int rc = recycle_check(r, force, s)) return rc;
    hipError_t e = launch_segment(d_events, nEvents, maxPacketsPerEvent, lbHdrVersion, maxPldLen, d_packets, stride,
                                  d_lens, s, nullptr, &r->dev, force != 0);
    if (e == hipSuccess) e = note_launch(r, s);
    if (e != hipSuccess) return hip_fail(e, "seg_kernel + recycle launch");
    return E2SAR_HIP_OK;
}

int e2sar_hip_reas_compact(e2sar_hip_reas *r, void *stream)
{
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    std::lock_guard<std::mutex> lk(r->mu);
    if (!r->alt.slots) return fail(E2SAR_HIP_ERR_LOGIC, "reassembler was not created COMPACTABLE");
    HIP_TRY(hipSetDevice(r->ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->ctx->stream;
    ReasCtl c;
    if (int rc = wait_launches(r)) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipMemcpy(&c, r->dev.ctl, sizeof(ReasCtl), hipMemcpyDeviceToHost));
    if (c.nCompleted != 0) return fail(E2SAR_HIP_ERR_LOGIC, "completed events not yet polled");
    hipError_t e = launch_compact(r->dev, r->alt, s);
    if (e == hipSuccess) e = note_launch(r, s);
    if (e != hipSuccess) return hip_fail(e, "compact launch");
    std::swap(r->dev.slots, r->alt.slots);
    std::swap(r->dev.arena, r->alt.arena);
    return E2SAR_HIP_OK;
}

int e2sar_hip_reas_reset_stats(e2sar_hip_reas *r, void *stream)
{
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    std::lock_guard<std::mutex> lk(r->mu);
    HIP_TRY(hipSetDevice(r->ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->ctx->stream;
    // the event counters (eventSuccess .. reassemblyLoss), the per-packet shards and the
    // error flags; the completed / lost records not yet polled stay queued (resetting
    // statistics in the reference discards no queued event), and so does inProgress, which
    // counts live table entries, not history
    auto *ctl = reinterpret_cast<uint8_t *>(r->dev.ctl);
    // kernels, not memset nodes: this call may be captured into a HIP graph
    HIP_TRY(launch_zero_words(ctl + offsetof(ReasCtl, eventSuccess),
                              (offsetof(ReasCtl, inProgress) - offsetof(ReasCtl, eventSuccess)) / 4, s));
    HIP_TRY(launch_zero_words(r->dev.shards, sizeof(ReasShard) * kShards / 4, s));
    HIP_TRY(launch_zero_words(ctl + offsetof(ReasCtl, errorFlags), 1, s));
    HIP_TRY(note_launch(r, s));
    return E2SAR_HIP_OK;
}

size_t e2sar_hip_route_workspace_bytes(uint32_t nPackets, uint32_t world)
{
    return route_workspace_bytes(nPackets, world);
}

}  // extern "C"

static int route(e2sar_hip_ctx *ctx, const uint8_t *d_packets, uint32_t stride, const uint32_t *d_lens,
                 uint32_t nPackets, int withLBHeader, uint32_t world, uint32_t self, int excludeSelf,
                 uint8_t *d_sendPackets, uint32_t *d_sendLens, uint32_t *d_counts, void *d_workspace,
                 size_t workspaceBytes, void *stream)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    if (world == 0 || world > 64 || self >= world) return fail(E2SAR_HIP_ERR_PARAMETER, "world must be 1..64, self < world");
    if ((stride & 15u) || stride < 48u) return fail(E2SAR_HIP_ERR_PARAMETER, "stride must be a multiple of 16, >= 48");
    if (nPackets && (!d_packets || !d_lens || !d_sendPackets || !d_sendLens || !d_counts || !d_workspace))
        return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer");
    if (workspaceBytes < route_workspace_bytes(nPackets, world)) return fail(E2SAR_HIP_ERR_PARAMETER, "workspace too small");
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    hipError_t e = launch_route(d_packets, stride, d_lens, nPackets, withLBHeader, world, self, excludeSelf,
                                d_sendPackets, d_sendLens, d_counts, d_workspace, s);
    if (e != hipSuccess) return hip_fail(e, "route launch");
    return E2SAR_HIP_OK;
}

extern "C" {

int e2sar_hip_route_batch(e2sar_hip_ctx *ctx, const uint8_t *d_packets, uint32_t stride, const uint32_t *d_lens,
                          uint32_t nPackets, int withLBHeader, uint32_t world, uint32_t self, uint8_t *d_sendPackets,
                          uint32_t *d_sendLens, uint32_t *d_counts, void *d_workspace, size_t workspaceBytes,
                          void *stream)
{
    return route(ctx, d_packets, stride, d_lens, nPackets, withLBHeader, world, self, 0, d_sendPackets, d_sendLens,
                 d_counts, d_workspace, workspaceBytes, stream);
}

int e2sar_hip_route_foreign(e2sar_hip_ctx *ctx, const uint8_t *d_packets, uint32_t stride, const uint32_t *d_lens,
                            uint32_t nPackets, int withLBHeader, uint32_t world, uint32_t self,
                            uint8_t *d_sendPackets, uint32_t *d_sendLens, uint32_t *d_counts, void *d_workspace,
                            size_t workspaceBytes, void *stream)
{
    return route(ctx, d_packets, stride, d_lens, nPackets, withLBHeader, world, self, 1, d_sendPackets, d_sendLens,
                 d_counts, d_workspace, workspaceBytes, stream);
}

int e2sar_hip_route_append(e2sar_hip_ctx *ctx, const uint8_t *d_packets, uint32_t stride, const uint32_t *d_lens,
                           uint32_t nPackets, int withLBHeader, uint32_t world, uint32_t self, int foreignOnly,
                           uint8_t *d_sendPackets, uint32_t *d_sendLens, uint32_t capPerRank, uint32_t *d_running,
                           void *d_workspace, size_t workspaceBytes, void *stream)
{
    if (!ctx) return fail(E2SAR_HIP_ERR_PARAMETER, "ctx is NULL");
    if (world == 0 || world > 64 || self >= world) return fail(E2SAR_HIP_ERR_PARAMETER, "world must be 1..64, self < world");
    if ((stride & 15u) || stride < 48u) return fail(E2SAR_HIP_ERR_PARAMETER, "stride must be a multiple of 16, >= 48");
    if (capPerRank == 0 || (uint64_t)capPerRank * world > 0xFFFFFFFFull)
        return fail(E2SAR_HIP_ERR_PARAMETER, "capPerRank must be > 0 and capPerRank * world < 2^32");
    if (!d_running) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL running counters");
    if (nPackets && (!d_packets || !d_lens || !d_sendPackets || !d_sendLens))
        return fail(E2SAR_HIP_ERR_PARAMETER, "NULL device buffer");
    (void)d_workspace;
    (void)workspaceBytes;                  // one launch, no workspace (kept in the signature for callers)
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    hipError_t e = launch_route_append(d_packets, stride, d_lens, nPackets, withLBHeader, world, self, foreignOnly ? 1 : 0,
                                       d_sendPackets, d_sendLens, capPerRank, d_running, s);
    if (e != hipSuccess) return hip_fail(e, "route launch");
    return E2SAR_HIP_OK;
}

int e2sar_hip_reas_set_owner(e2sar_hip_reas *r, uint32_t world, uint32_t self)
{
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    if (world == 0 || world > 64 || self >= world) return fail(E2SAR_HIP_ERR_PARAMETER, "world must be 1..64, self < world");
    std::lock_guard<std::mutex> lk(r->mu);
    r->dev.ownWorld = r->alt.ownWorld = world;
    r->dev.ownSelf = r->alt.ownSelf = self;
    return E2SAR_HIP_OK;
}

int e2sar_hip_reas_forget_stream(e2sar_hip_reas *r, void *stream)
{
    if (!r || !stream) return fail(E2SAR_HIP_ERR_PARAMETER, "NULL argument");
    std::lock_guard<std::mutex> lk(r->mu);
    HIP_TRY(hipSetDevice(r->ctx->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    HIP_TRY(hipStreamSynchronize(s));
    r->streams.erase(s);
    drop_scratch(r, s);
    return E2SAR_HIP_OK;
}

int e2sar_hip_reas_set_cold(e2sar_hip_reas *r, int cold)
{
    if (!r) return fail(E2SAR_HIP_ERR_PARAMETER, "reas is NULL");
    std::lock_guard<std::mutex> lk(r->mu);
    if (cold) r->cfg.flags |= E2SAR_HIP_REAS_COLD_DATAGRAMS;
    else r->cfg.flags &= ~E2SAR_HIP_REAS_COLD_DATAGRAMS;
    return E2SAR_HIP_OK;
}

}  // extern "C"
