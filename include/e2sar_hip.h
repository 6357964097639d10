/*
 * e2sar_hip.h -- C ABI of the MI355X (gfx950) SAR data path.
 *
 * This is the drop-in boundary for the reference's segmentation / reassembly hot path
 * (JeffersonLab/E2SAR v0.3.2).  Plain C: pointers, sizes, integer status codes; no HIP,
 * torch or C++ types cross it.  Device pointers are passed as ordinary pointers that
 * were allocated on the context's device (hipMalloc, torch, or e2sar_hip_device_alloc).
 *
 * Each entry point names the reference interface it replaces (file:line).
 *
 * Status codes: 0 = success, negative = -(E2SARErrorc) from include/e2sarError.hpp:23-39
 * (e.g. -3 ParameterError, -5 OutOfRange, -7 NotFound, -10 MemoryError, -11 LogicError,
 * -12 SystemError for a HIP runtime failure, -13 DataError).  No C++ exception crosses
 * this boundary (the reference methods are noexcept, e2sarDPSegmenter.hpp:458-483).
 */
#ifndef E2SAR_HIP_H
#define E2SAR_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define E2SAR_HIP_ABI_VERSION 1

enum {
    E2SAR_HIP_OK = 0,
    E2SAR_HIP_ERR_PARAMETER = -3,   /* E2SARErrorc::ParameterError */
    E2SAR_HIP_ERR_OUT_OF_RANGE = -5,/* E2SARErrorc::OutOfRange */
    E2SAR_HIP_ERR_NOT_FOUND = -7,   /* E2SARErrorc::NotFound */
    E2SAR_HIP_ERR_MEMORY = -10,     /* E2SARErrorc::MemoryError */
    E2SAR_HIP_ERR_LOGIC = -11,      /* E2SARErrorc::LogicError */
    E2SAR_HIP_ERR_SYSTEM = -12,     /* E2SARErrorc::SystemError (HIP runtime failure) */
    E2SAR_HIP_ERR_DATA = -13        /* E2SARErrorc::DataError */
};

/* LB+RE header geometry on the wire (e2sarHeaders.hpp:302-315): 16-byte LB + 20-byte RE */
#define E2SAR_HIP_LB_HDR_LEN 16
#define E2SAR_HIP_RE_HDR_LEN 20
#define E2SAR_HIP_LBRE_HDR_LEN 36

/* ------------------------------------------------------------------ */
/* library / context                                                   */

int e2sar_hip_abi_version(void);
/* Human-readable message for the last failing call on this thread (E2SARErrorInfo::msg). */
const char *e2sar_hip_last_error(void);

typedef struct e2sar_hip_ctx e2sar_hip_ctx;
/* Bind a device and a stream.  `stream` is the hipStream_t every call of this context
 * runs on when the call's own `stream` argument is NULL; NULL here means the device's
 * default stream.  Replaces the per-Segmenter/Reassembler thread state
 * (e2sarDPSegmenter.hpp:213-260, e2sarDPReassembler.hpp:206-240): one context per
 * sending/receiving thread gives the same concurrency without shared mutable state. */
int e2sar_hip_ctx_create(int device, void *stream, e2sar_hip_ctx **out);
/* A non-blocking stream for callers without a HIP toolchain. */
int e2sar_hip_stream_create(int device, void **out);
int e2sar_hip_stream_destroy(void *stream);
/* Every reassembler created on a context holds a reference to it: a context and its
 * reassemblers may be destroyed in any order (the memory goes with the last of them). */
void e2sar_hip_ctx_destroy(e2sar_hip_ctx *ctx);
void *e2sar_hip_ctx_stream(e2sar_hip_ctx *ctx);
int e2sar_hip_ctx_device(e2sar_hip_ctx *ctx);
int e2sar_hip_ctx_sync(e2sar_hip_ctx *ctx);

/* memory plumbing so callers without a HIP toolchain (cgo/ctypes/C++) can drive the path */
int e2sar_hip_device_alloc(e2sar_hip_ctx *ctx, size_t bytes, void **out);
int e2sar_hip_device_free(e2sar_hip_ctx *ctx, void *p);
int e2sar_hip_host_alloc(size_t bytes, void **out);           /* pinned host memory */
int e2sar_hip_host_free(void *p);
int e2sar_hip_memcpy_h2d(e2sar_hip_ctx *ctx, void *dst, const void *src, size_t bytes);
int e2sar_hip_memcpy_d2h(e2sar_hip_ctx *ctx, void *dst, const void *src, size_t bytes);
/* fill `bytes` device bytes with (uint8_t)value on the context stream: a kernel, not
 * hipMemsetAsync, so the call may be captured into a HIP graph (captured memset nodes write
 * garbage from the second replay on with this ROCm) */
int e2sar_hip_memset_d(e2sar_hip_ctx *ctx, void *dst, int value, size_t bytes);
/* e2sar_hip_memset_d on `stream` (NULL = context stream): a fill kernel, capture-safe */
int e2sar_hip_memset_async(e2sar_hip_ctx *ctx, void *dst, int value, size_t bytes, void *stream);
/* asynchronous copy on `stream` (NULL = context stream); kind 0 = H2D, 1 = D2H, 2 = D2D */
int e2sar_hip_memcpy_async(e2sar_hip_ctx *ctx, void *dst, const void *src, size_t bytes, int kind,
                           void *stream);
int e2sar_hip_stream_sync(e2sar_hip_ctx *ctx, void *stream);

/* stream ordering for callers without a HIP toolchain (the C++ facade pipelines its
 * host->device copies beside the reassembly kernels with these): an event records the
 * point a stream has reached; another stream can wait for it, the host can query or wait. */
int e2sar_hip_event_create(e2sar_hip_ctx *ctx, void **out);
int e2sar_hip_event_destroy(void *event);
int e2sar_hip_event_record(e2sar_hip_ctx *ctx, void *event, void *stream);   /* NULL stream = context stream */
int e2sar_hip_stream_wait_event(e2sar_hip_ctx *ctx, void *stream, void *event);
int e2sar_hip_event_query(void *event);        /* 1 = reached, 0 = not yet, < 0 = error */
int e2sar_hip_event_sync(void *event);

/* Gather copy: n spans {src, dst, bytes}, device or pinned host memory on either side
 * (pinned memory from e2sar_hip_host_alloc is device-accessible at the same address), in
 * one kernel launch per 64 spans on `stream`.  This is how completed events leave the
 * device arena in one batch instead of one memcpy per event. */
typedef struct e2sar_hip_copy_span {
    const void *src;
    void *dst;
    uint64_t bytes;
} e2sar_hip_copy_span;
int e2sar_hip_copy_spans(e2sar_hip_ctx *ctx, const e2sar_hip_copy_span *spans, uint32_t n, void *stream);

/* ------------------------------------------------------------------ */
/* geometry (e2sarHeaders.hpp:415-421, e2sarDPSegmenter.hpp:241, e2sarDPSegmenter.cpp:670) */

size_t e2sar_hip_total_hdr_len(int useIPv6);                 /* 64 (v4) / 84 (v6) */
size_t e2sar_hip_max_pld_len(uint32_t mtu, int useIPv6);     /* mtu - total_hdr_len; 0 if mtu too small */
size_t e2sar_hip_num_packets(size_t bytes, size_t maxPldLen);/* ceil(bytes / maxPldLen) */
/* device packet slot: 36 + maxPldLen rounded up to 16 bytes */
uint32_t e2sar_hip_packet_stride(size_t maxPldLen);

/* ------------------------------------------------------------------ */
/* segmentation: replaces SendThreadState::_send's fragment loop        */
/* (e2sarDPSegmenter.cpp:660-871) for a batch of events                 */

/* One event: the arguments of _send (cpp:660-662) after the host has applied the
 * event-numbering rule (cpp:901-917 / 920-948), the dataId default (cpp:938), entropy
 * "0 => random" (cpp:727-728), the LB tick (cpp:707-719) and ticksAsREEventNum
 * (cpp:723-724).  40 bytes, 8-byte aligned. */
typedef struct e2sar_hip_seg_event {
    const uint8_t *data;   /* device address of the event bytes */
    uint64_t eventNum;     /* RE eventNum */
    uint64_t lbTick;       /* LB eventNum (v2) / tick (v3) */
    uint32_t bytes;        /* event length; REHdr bufferLength is u32 (e2sarHeaders.hpp:26) */
    uint32_t pktBase;      /* index of the event's first packet in the batch (set by seg_plan) */
    uint16_t dataId;
    uint16_t entropy;
    uint32_t reserved;
} e2sar_hip_seg_event;

/* Host-side plan over a host copy of the event table: fills pktBase (exclusive prefix
 * of ceil(bytes/maxPldLen)) and writes the batch's packet count and the largest per-event
 * packet count to *totalPackets and *maxPacketsPerEvent (either may be NULL).  Returns a
 * status: 0, or E2SAR_HIP_ERR_PARAMETER (NULL table, maxPldLen 0) / OUT_OF_RANGE (more
 * than 2^32 - 1 packets). */
int e2sar_hip_seg_plan(e2sar_hip_seg_event *events, uint32_t nEvents, size_t maxPldLen,
                       uint32_t *totalPackets, uint32_t *maxPacketsPerEvent);

/* Segment nEvents events (descriptor table `d_events` already on the device) into
 * datagrams [16-byte LB][20-byte RE][payload] at d_packets + p*stride, p = pktBase+k.
 * d_lens[p] (optional) receives the datagram length 36 + payload.  lbHdrVersion 3
 * selects LBHdrV3, any other value LBHdrV2 (e2sarHeaders.hpp:287-297).
 * maxPacketsPerEvent: an upper bound (from seg_plan).  eventsDwordAligned is a hint kept
 * for ABI compatibility: the kernel takes its 16-byte dword-aligned fast path for every
 * event whose address and maxPldLen are multiples of 4 and a byte path for the others,
 * checking each event itself.  Asynchronous on `stream` (NULL = the context stream). */
int e2sar_hip_segment_batch(e2sar_hip_ctx *ctx, const e2sar_hip_seg_event *d_events,
                            uint32_t nEvents, uint32_t maxPacketsPerEvent,
                            int lbHdrVersion, uint32_t maxPldLen, int eventsDwordAligned,
                            uint8_t *d_packets, uint32_t stride, uint32_t *d_lens,
                            void *stream);

/* ------------------------------------------------------------------ */
/* reassembly: replaces the RecvThreadState per-packet body             */
/* (e2sarDPReassembler.cpp:310-428), eventsInProgress (hpp:224-233),    */
/* the event queue (hpp:126-161) and the GC pass (cpp:236-291)          */

typedef struct e2sar_hip_reas e2sar_hip_reas;

typedef struct e2sar_hip_reas_config {
    int withLBHeader;          /* ReassemblerFlags::withLBHeader (hpp:436) */
    uint32_t tableSlots;       /* in-progress event table slots (power of two, >= 64) */
    uint32_t queueCapacity;    /* completed-event records held until polled (QSIZE, hpp:126) */
    uint32_t lostCapacity;     /* lost-event records held until polled */
    uint64_t arenaBytes;       /* device arena that receives reassembled event bytes */
    uint32_t flags;            /* E2SAR_HIP_REAS_* */
    uint32_t groupSize;        /* datagrams per workgroup of the fused reassembly kernel (1..64);
                                  0 = automatic: a 9K-chunk budget balanced to whole residency
                                  waves of the chip (the measured best) */
} e2sar_hip_reas_config;

/* Allocate a second table + arena so e2sar_hip_reas_compact() can move in-progress
 * events out of a full arena (streaming use: events that straddle batches). */
#define E2SAR_HIP_REAS_COMPACTABLE 1u
/* Reassemble with the reference receive body's arrival-order rules, whatever the order:
 * a fragment with bufferOffset 0 always starts a new item, dropping an item in progress
 * under the same (eventNum, dataId) without a lost record (e2sarDPReassembler.cpp:361-369);
 * a fragment whose key has no item starts one, also after its event completed
 * (cpp:376-384); completion is tested after every fragment (cpp:403), so duplicates
 * before the last fragment overshoot curBytes.  Arrival order = batch order, then datagram
 * order in the batch.  Without the flag the device path is order-insensitive: every
 * fragment joins its event and completion is tested per run of a launch (identical results
 * whenever offset 0 arrives first and there are no duplicates).  The mode
 * adds a key pass and a per-key walk per batch and device scratch (about 56 bytes per
 * datagram of the largest batch, 48 more in reassemble_batch for its work records, and 524
 * bytes per table slot) that grows on demand (per stream; it cannot
 * grow inside a graph capture -- such a launch fails with LOGIC -- so capture only after a
 * first batch of the largest size has run on the capturing stream). */
#define E2SAR_HIP_REAS_REFERENCE_ORDER 2u
/* The datagram batches of this reassembler were written long before they are reassembled
 * (not in the Infinity Cache, e.g. received into HBM well ahead): the split, pipelined and
 * reference-order forms read them with streaming (non-temporal) loads.  Without the flag
 * they use cache-allocating loads (a batch just written -- by the segmenter, a copy, the NIC
 * -- is read from cache), except for batches above 320 MiB of slots, which cannot be. */
#define E2SAR_HIP_REAS_COLD_DATAGRAMS 4u

/* Reassembled event handed to the caller (getEvent's out-params, cpp:626-641).
 * The bytes live at e2sar_hip_reas_arena() + arenaOffset until the arena is recycled. */
typedef struct e2sar_hip_event_rec {
    uint64_t eventNum;
    uint64_t arenaOffset;
    uint32_t bytes;
    uint16_t dataId;
    uint16_t flags;
    uint32_t numFragments;
    uint32_t reserved;
} e2sar_hip_event_rec;

/* get_LostEvent's tuple (hpp:593-604) + which loss it was. */
typedef struct e2sar_hip_lost_rec {
    uint64_t eventNum;
    uint64_t numFragments;
    uint16_t dataId;
    uint16_t enqueueLoss;      /* 1 = lost on enqueue (queue/arena full), 0 = reassembly (GC) */
    uint32_t reserved;
} e2sar_hip_lost_rec;

/* Reassembler::ReportedStats (hpp:383-400) plus device-path diagnostics. */
typedef struct e2sar_hip_reas_stats {
    uint64_t enqueueLoss;
    uint64_t reassemblyLoss;
    uint64_t eventSuccess;
    uint64_t totalPackets;
    uint64_t totalBytes;
    uint64_t badHeaderDiscards;
    uint64_t dataErrCnt;
    int64_t inProgress;
    uint64_t completedPending;   /* records waiting in the completion list */
    uint64_t lostPending;
    uint64_t arenaUsed;
    uint64_t tableUsed;          /* slots ever claimed since the last recycle */
    uint32_t errorFlags;         /* bit0 table full, bit1 arena full, bit2 probe timeout,
                                    bit3 scatter record outside the arena (bad work buffer),
                                    bit4 chained form: a group's datagrams never all written
                                    (wait timed out), bit5 chained form: counter over-count */
    uint32_t reserved;
} e2sar_hip_reas_stats;

int e2sar_hip_reas_create(e2sar_hip_ctx *ctx, const e2sar_hip_reas_config *cfg,
                          e2sar_hip_reas **out);
void e2sar_hip_reas_destroy(e2sar_hip_reas *r);
/* device base of the event arena */
uint8_t *e2sar_hip_reas_arena(e2sar_hip_reas *r);

/* Parse, validate, look up / create and scatter nPackets datagrams held at
 * d_packets + p*stride with lengths d_lens[p] (the full datagram length as recvfrom
 * returns it, cpp:321).  now_ms stamps firstSegment for new events (hpp:97).
 * One fused launch for batches of up to 320 MiB of slots; above that (a batch that cannot
 * sit in the Infinity Cache) classify + scatter launches through an internal work buffer.
 * Internal buffers (this form, reference order) are kept per stream, so batches may be launched on several streams at once; they grow on first
 * use for a size, never inside a graph capture (LOGIC error: run one batch of the largest
 * size on the stream first), and an outgrown buffer stays allocated until destroy, so a
 * graph captured earlier keeps valid addresses.
 * Asynchronous on `stream` (NULL = the context stream). */
int e2sar_hip_reassemble_batch(e2sar_hip_reas *r, const uint8_t *d_packets, uint32_t stride,
                               const uint32_t *d_lens, uint32_t nPackets, uint64_t now_ms,
                               void *stream);

/* The same work as e2sar_hip_reassemble_batch split in two phases so a caller can
 * pipeline batches: classify (headers only: validate, look up / create, count) writes
 * per-datagram destinations into d_work; scatter moves the payload bytes and publishes
 * the events the batch completed.  Scatter a batch after its classify (same packets,
 * stride, nPackets and work buffer, ordered on one stream or by an event); the work
 * buffer is reusable once that scatter has run.  Batches are classified in arrival order.
 * d_work: device memory, 256-byte aligned, e2sar_hip_reas_work_bytes(nPackets) bytes;
 * no initialisation needed.  Asynchronous.  Replaces the same per-packet body
 * (e2sarDPReassembler.cpp:335-427) as e2sar_hip_reassemble_batch. */
size_t e2sar_hip_reas_work_bytes(uint32_t nPackets);
int e2sar_hip_reas_classify(e2sar_hip_reas *r, const uint8_t *d_packets, uint32_t stride,
                            const uint32_t *d_lens, uint32_t nPackets, uint64_t now_ms,
                            void *d_work, size_t workBytes, void *stream);
int e2sar_hip_reas_scatter(e2sar_hip_reas *r, const uint8_t *d_packets, uint32_t stride,
                           uint32_t nPackets, const void *d_work, size_t workBytes, void *stream);
/* Pipelined step, one launch: scatter the classified batch b (d_spk, sn, d_swork) while
 * other workgroups of the same grid classify batch b+1 (d_cpk, d_clens, cn, d_cwork).
 * The two batches use different packet and work buffers.  A stream of batches runs as
 * classify(0), scatter_classify(0, 1), ..., scatter_classify(k-1, k), scatter(k). */
int e2sar_hip_reas_scatter_classify(e2sar_hip_reas *r, uint32_t stride,
                                    const uint8_t *d_spk, uint32_t sn, const void *d_swork,
                                    size_t sworkBytes, const uint8_t *d_cpk,
                                    const uint32_t *d_clens, uint32_t cn, uint64_t now_ms,
                                    void *d_cwork, size_t cworkBytes, void *stream);

/* GC pass: events whose first fragment is older than timeout_ms become lost
 * (reassemblyLoss, cpp:252-274).  Asynchronous. */
int e2sar_hip_reas_gc(e2sar_hip_reas *r, uint64_t now_ms, uint64_t timeout_ms, void *stream);

/* Drain completed events.  Waits, under the reassembler's lock, for every kernel launched
 * through this reassembler (an event recorded after each launch on each stream used; other
 * streams and reassemblers are not waited for), so none runs while the list is drained.
 * Once a launch of this reassembler has been captured into a HIP graph, replays may run on
 * any stream and the wait covers the whole device.  Records are returned in completion
 * order of the device; *nOut <= cap.  Records beyond cap stay queued. */
int e2sar_hip_reas_poll(e2sar_hip_reas *r, e2sar_hip_event_rec *out, uint32_t cap,
                        uint32_t *nOut);
/* Drain lost-event records (waits for this reassembler's launches, as reas_poll). */
int e2sar_hip_reas_lost_poll(e2sar_hip_reas *r, e2sar_hip_lost_rec *out, uint32_t cap,
                             uint32_t *nOut);
/* Stats snapshot (waits for this reassembler's launches, as reas_poll). */
int e2sar_hip_reas_get_stats(e2sar_hip_reas *r, e2sar_hip_reas_stats *out);
/* Recycle the arena and the event table.  Only legal when no event is in progress
 * and every completed record has been polled (else E2SAR_HIP_ERR_LOGIC); the caller
 * promises it no longer reads event bytes from the arena.  `force` drops in-progress
 * events without logging them.  Asynchronous. */
int e2sar_hip_reas_recycle(e2sar_hip_reas *r, int force, void *stream);
/* e2sar_hip_segment_batch and e2sar_hip_reas_recycle(r, force) in ONE launch: extra
 * workgroups at the end of the segmentation grid reset r's table and arena (no seg block
 * touches them).  Same preconditions as the two calls; r's earlier launches on `stream`
 * finish before it starts, and its next reassembly starts after it.  What it saves is one
 * launch and its boundary per step (the bench's step: recycle, then segment -> reassemble
 * per batch).  Replaces nothing in the reference (whose events are new[] buffers); see
 * e2sar_hip_reas_recycle. */
int e2sar_hip_segment_batch_recycle(e2sar_hip_ctx *ctx, const e2sar_hip_seg_event *d_events, uint32_t nEvents,
                                    uint32_t maxPacketsPerEvent, int lbHdrVersion, uint32_t maxPldLen,
                                    int eventsDwordAligned, uint8_t *d_packets, uint32_t stride, uint32_t *d_lens,
                                    e2sar_hip_reas *r, int force, void *stream);
/* Streaming form of recycle: move every in-progress event (its table entry and the
 * bytes received so far) to the alternate table/arena, which becomes current; the old
 * arena is free again.  Needs E2SAR_HIP_REAS_COMPACTABLE, and every completed record
 * polled (their arena offsets refer to the old arena; copy the bytes out first).
 * Asynchronous; e2sar_hip_reas_arena() returns the new base afterwards. */
int e2sar_hip_reas_compact(e2sar_hip_reas *r, void *stream);
/* Zero the statistics counters (event counters, per-datagram counters, error flags).
 * Completed and lost records not yet polled stay queued.  Asynchronous. */
int e2sar_hip_reas_reset_stats(e2sar_hip_reas *r, void *stream);

/* ------------------------------------------------------------------ */
/* relay (BASELINE config 5: receive -> reassemble -> segment -> send on one GPU): the    */
/* events a reassembler completed are segmented again without a host round trip.  The  */
/* Segmenter's per-event rules (numbering, dataId, entropy, LB tick: cpp:707-728,      */
/* 901-948) are replaced by: RE eventNum and dataId as received, one LB tick for the   */
/* batch, entropy of the i-th planned event = entropyBase + i (mod 2^16).               */

/* Completed records [firstRecord, firstRecord + n) -- n = min(maxEvents, records the    */
/* reassembler holds past firstRecord) -- become seg descriptors d_events[0, n) (device, */
/* maxEvents entries) with pktBase filled in; d_counts[0] = n, d_counts[1] = their       */
/* datagram count (device, 2 entries).  The event bytes stay in the arena: recycle or    */
/* compact only after the segmentation that reads them.  Asynchronous.                  */
int e2sar_hip_relay_plan(e2sar_hip_reas *r, uint32_t firstRecord, uint32_t maxEvents, size_t maxPldLen,
                         uint64_t lbTick, uint16_t entropyBase, e2sar_hip_seg_event *d_events,
                         uint32_t *d_counts, void *stream);
/* e2sar_hip_segment_batch with the event count read on the device (d_counts[0], as     */
/* e2sar_hip_relay_plan writes it); maxEvents bounds it.  Event data 256-byte aligned    */
/* (arena buffers), so the dword-aligned path is used when maxPldLen % 4 == 0.           */
int e2sar_hip_segment_batch_dev(e2sar_hip_ctx *ctx, const e2sar_hip_seg_event *d_events,
                                const uint32_t *d_counts, uint32_t maxEvents, uint32_t maxPacketsPerEvent,
                                int lbHdrVersion, uint32_t maxPldLen, uint8_t *d_packets, uint32_t stride,
                                uint32_t *d_lens, void *stream);

/* ------------------------------------------------------------------ */
/* multi-GPU: events are owned by rank eventNum % world.  A rank that received       */
/* (landed) datagrams of other ranks' events routes them: this packs the batch into */
/* per-destination spans (stable order) and reports the span sizes, ready for one   */
/* all-to-all-v over RCCL.  The reference never needs this step: its load balancer  */
/* steers every fragment of an event to one receiver (e2sarDPSegmenter.hpp:231-235). */

size_t e2sar_hip_route_workspace_bytes(uint32_t nPackets, uint32_t world);
/* d_sendPackets: nPackets*stride bytes; d_sendLens: nPackets; d_counts: world entries
 * (datagrams per destination rank).  Datagrams whose RE header does not parse stay on
 * `self`.  world <= 64.  Asynchronous. */
int e2sar_hip_route_batch(e2sar_hip_ctx *ctx, const uint8_t *d_packets, uint32_t stride,
                          const uint32_t *d_lens, uint32_t nPackets, int withLBHeader,
                          uint32_t world, uint32_t self, uint8_t *d_sendPackets,
                          uint32_t *d_sendLens, uint32_t *d_counts, void *d_workspace,
                          size_t workspaceBytes, void *stream);
/* Foreign-only routing: as e2sar_hip_route_batch, but datagrams this rank keeps -- owned
 * by `self`, or unparsable -- are neither packed nor counted (d_counts[self] = 0, and no
 * byte of theirs is read beyond the RE header).  They are reassembled where they landed
 * by a reassembler set to this rank's ownership (e2sar_hip_reas_set_owner), so only
 * (world-1)/world of an evenly spread batch crosses HBM twice and xGMI once.  Asynchronous. */
int e2sar_hip_route_foreign(e2sar_hip_ctx *ctx, const uint8_t *d_packets, uint32_t stride,
                            const uint32_t *d_lens, uint32_t nPackets, int withLBHeader,
                            uint32_t world, uint32_t self, uint8_t *d_sendPackets,
                            uint32_t *d_sendLens, uint32_t *d_counts, void *d_workspace,
                            size_t workspaceBytes, void *stream);

/* Per-batch routing into per-rank regions, for a stream of landed batches exchanged once
 * per step: rank d's datagrams are appended to region d -- slots [d*capPerRank,
 * (d+1)*capPerRank) of d_sendPackets / d_sendLens -- after the ones already there, and
 * running[d] (device, world counters, zeroed by the caller before the first batch, e.g.
 * e2sar_hip_memset_d) grows by this batch's count for d.  One launch: each workgroup of 256
 * datagrams reserves its room with one atomic per destination, so within a batch the order
 * of a destination's datagrams is kept inside each 256-datagram block, and the blocks
 * append in the order they reserve (the order-insensitive reassembler does not care; a
 * REFERENCE_ORDER receiver takes the region order as the arrival order).  The workspace
 * arguments are unused (NULL / 0 allowed).  A datagram that would land past
 * its region is not written, but still counted: running[d] > capPerRank after the step
 * means the regions were too small.  foreignOnly: as e2sar_hip_route_foreign (this rank's
 * datagrams and unparsable ones stay here, running[self] stays 0).  Routing each batch
 * right after it landed reads it while it is still in the Infinity Cache; the step's one
 * all-to-all then sends each region's first running[d] slots.  Asynchronous. */
int e2sar_hip_route_append(e2sar_hip_ctx *ctx, const uint8_t *d_packets, uint32_t stride,
                           const uint32_t *d_lens, uint32_t nPackets, int withLBHeader,
                           uint32_t world, uint32_t self, int foreignOnly, uint8_t *d_sendPackets,
                           uint32_t *d_sendLens, uint32_t capPerRank, uint32_t *d_running,
                           void *d_workspace, size_t workspaceBytes, void *stream);

/* Ownership of a reassembler in a world of `world` ranks (1..64): from the next launch on,
 * a datagram whose RE header parses but whose eventNum % world != self belongs to another
 * rank and takes no part -- not counted in any statistic, no byte copied.  Unparsable
 * datagrams are still counted (badHeaderDiscards) here.  world = 1 (the default) takes
 * every datagram.  The receive-side counterpart of the reference's steering of every
 * fragment of an event to one receiver by eventNum (e2sarDPReassembler.hpp:224-229). */
int e2sar_hip_reas_set_owner(e2sar_hip_reas *r, uint32_t world, uint32_t self);
/* Set (cold != 0) or clear E2SAR_HIP_REAS_COLD_DATAGRAMS for the following launches: a
 * reassembler that takes both just-written and long-resident batches (e.g. datagrams
 * reassembled where they landed, then datagrams received from other ranks) tells each
 * launch how to load them. */
int e2sar_hip_reas_set_cold(e2sar_hip_reas *r, int cold);
/* Before destroying a stream that launched through this reassembler: wait for the stream's
 * work, stop tracking it and free its internal buffers (or retire them, if a launch of this
 * reassembler was ever captured).  Snapshots (poll, lost_poll, get_stats) wait for every
 * stream the reassembler launched on, so a stream must outlive the reassembler's last
 * snapshot unless it is forgotten first: HIP may hand a destroyed stream's handle to a new
 * stream.  (A snapshot that finds a handle already invalid drops it the same way.)  The
 * stream must still be alive when this is called (it is synchronised): call it, then
 * destroy the stream -- never the other way round.  No reference counterpart: the
 * reference's receive threads own their sockets for their life. */
int e2sar_hip_reas_forget_stream(e2sar_hip_reas *r, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* E2SAR_HIP_H */
