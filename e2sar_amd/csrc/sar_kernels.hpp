// sar_kernels.hpp -- device data layout and launchers of the gfx950 SAR path.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "e2sar_hip.h"

// launch forms kept for A/B only (include/e2sar_hip_experimental.h; `make experimental`)
#ifndef E2SAR_HIP_EXPERIMENTAL
#define E2SAR_HIP_EXPERIMENTAL 0
#endif

namespace e2sar_amd {

// In-progress event table entry (the device form of eventsInProgress's
// shared_ptr<EventQueueItem>, e2sarDPReassembler.hpp:61-99, 224-233).  64 bytes, in two
// 16-byte records a lookup reads in one round trip: A = {state, dataId, eventNum}, written
// by one 16-byte store when the slot is published, and B = {bufOff, bytes, bvalid}.
struct ReasSlot {
    uint32_t state;      // EMPTY / BUSY / READY / DONE / LOST
    uint32_t dataId;
    uint64_t eventNum;
    uint64_t bufOff;     // arena offset of the event buffer
    uint32_t bytes;      // bufferLength of the packet that created the event
    uint32_t bvalid;     // 1 once bufOff/bytes are written
    unsigned long long acc;  // curBytes (low 36 bits) | numFragments (high 28 bits)
    uint64_t created;    // firstSegment, caller clock in ms
    uint64_t pad1[2];
};
static_assert(sizeof(ReasSlot) == 64, "slot is one 64-byte line");
static_assert(offsetof(ReasSlot, eventNum) == 8 && offsetof(ReasSlot, bufOff) == 16 && offsetof(ReasSlot, bvalid) == 28,
              "records A and B are the two first 16-byte quarters of the slot");

constexpr uint32_t kAccFragShift = 36;
constexpr uint64_t kAccBytesMask = (1ull << kAccFragShift) - 1ull;

// Per-event counters (Reassembler::AtomicStats, e2sarDPReassembler.hpp:102-122) + allocator
// state; the per-packet counters live in ReasShard.
struct ReasCtl {
    // every creator's returning atomic lands here: alone on its 128-byte line (A/B: +0.7 %)
    unsigned long long arenaTop;
    uint64_t padA[15];
    unsigned long long eventSuccess;
    unsigned long long enqueueLoss;
    unsigned long long reassemblyLoss;
    long long inProgress;
    uint32_t nCompleted;
    uint32_t nLost;
    uint32_t tableUsed;
    uint32_t errorFlags;
    unsigned long long compactTop;   // arena top of the destination arena during compaction
    uint32_t compactUsed;            // slots claimed in the destination table
    uint32_t pad0;
    uint64_t pad[2];
    uint64_t pad2[6];
};
static_assert(sizeof(ReasCtl) % 128 == 0, "shards follow the control block on 128-byte lines");

// Per-packet counters are sharded (one 128-byte line per shard, shard = block % kShards)
// so thousands of waves do not serialise on one address; the host sums the shards.
constexpr uint32_t kShards = 64;
struct ReasShard {
    unsigned long long totalPackets;
    unsigned long long totalBytes;
    unsigned long long badHeaderDiscards;
    unsigned long long dataErrCnt;
    unsigned long long eventSuccess;   // shard = slot % kShards; ReasCtl::eventSuccess stays 0
    unsigned long long pad[11];
};
static_assert(sizeof(ReasShard) == 128, "one shard per 128-byte line");

// Table-occupancy deltas, sharded the same way (shard = slot % kShards) on lines of their
// own after the ReasShard array: every creator and every completer used to hit
// ReasCtl::inProgress / tableUsed, which serialised small events (64 KiB / MTU 1500:
// 897 -> 1190 GiB/s with the two counters removed).  The live values are ReasCtl's base
// plus the sum over the shards; recycle and compaction, which re-base them, zero these too.
// reset_stats leaves them alone (they count live entries, not history).
struct ReasOcc {
    long long inProgress;
    long long tableUsed;
    uint64_t pad[14];
};
static_assert(sizeof(ReasOcc) == 128, "one occupancy shard per 128-byte line");

// Everything a reassembly kernel needs, passed by value.
struct ReasDev {
    ReasSlot *slots;
    ReasCtl *ctl;
    ReasShard *shards;
    e2sar_hip_event_rec *completed;
    e2sar_hip_lost_rec *lost;
    uint8_t *arena;
    uint64_t arenaBytes;
    uint32_t tableSlots;      // power of two
    uint32_t queueCapacity;
    uint32_t lostCapacity;
    int withLB;
    // multi-GPU ownership (e2sar_hip_reas_set_owner): with ownWorld > 1 a datagram whose RE
    // header parses but whose eventNum % ownWorld != ownSelf belongs to another rank and is
    // skipped -- neither counted nor copied (that rank's reassembler counts it)
    uint32_t ownWorld;
    uint32_t ownSelf;
    uint32_t groupSize;       // datagrams per reas_kernel workgroup (config), 0 = chip-balanced auto
};

// Per-datagram result of classification (held in LDS between the two phases of reas_kernel).
struct PktInfo {
    uint64_t dst;     // device address of the payload's destination (0 = drop)
    uint32_t plen;    // payload bytes
    uint32_t hl;      // header bytes in front of the payload (36 with LB header, else 20)
};
static_assert(sizeof(PktInfo) == 16, "one dwordx4 per packet");

// An event completed by a classified batch, published by the scatter kernel of that batch.
struct FinishRec {
    uint64_t ev;
    uint64_t boff;
    uint32_t slot;
    uint32_t bytes;
    uint32_t frags;
    uint32_t d;
};
static_assert(sizeof(FinishRec) == 32, "two dwordx4 per record");

// Work buffer of one classified batch of n datagrams (caller-owned, device memory):
//   [0, 16n)                  PktInfo per datagram
//   [work_fin_off(n), + 32n)  FinishRec per datagram (written only by completing run tails)
inline size_t work_fin_off(uint32_t n) { return ((size_t)n * sizeof(PktInfo) + 255) & ~(size_t)255; }
inline size_t work_bytes(uint32_t n) { return work_fin_off(n) + (size_t)n * sizeof(FinishRec); }

// Reference-order mode: per-datagram record of ro_key_kernel, and the scratch it needs for a
// batch of n datagrams and a table of T slots.  Round 5: no sort of the datagrams -- the key
// pass files every run of consecutive positions of one key into its slot's bucket of
// kRoBucket runs (past that into an overflow list, placed and sorted by ro_place_kernel), and
// each key's walk orders its own runs by position.
constexpr uint32_t kRoBucket = 64;
struct RoRec {
    uint32_t off, plen, blen, hl;
};
static_assert(sizeof(RoRec) == 16, "one dwordx4 per datagram");
struct RoRun {
    uint32_t slot, start, len, k;   // k: the run's index among its key's runs (the key pass's count)
};
static_assert(sizeof(RoRun) == 16, "one dwordx4 per run");
struct RoScratch {
    uint32_t *ctr;                  // [0] overflow flag, [1] keys with runs (both zero between batches),
                                    // [2] keys with runs for the walk
    uint32_t *runCnt;               // [T] runs per slot                        (zero between batches)
    uint32_t *runBase;              // [T] place of a slot of more than kRoBucket runs (runs k >= kRoBucket at + k)
    uint32_t *active;               // [T] slots with runs in this batch
    unsigned long long *bucket;     // [T][kRoBucket] start << 32 | len, in filing order
    RoRec *recs;                    // [n]
    RoRun *runs;                    // [n] overflow runs, at their head datagram's position
    unsigned long long *ovMask;     // [n / 64] per key-pass wave: lanes that head an overflow run
    unsigned long long *placed;     // [n] overflow runs of the slots of more than kRoBucket runs, by k
    unsigned long long *sortTmp;    // [2n] a slot's padded sort at 2 x runBase (slots of > 2048 runs)
};
inline size_t ro_align(size_t x) { return (x + 255) & ~(size_t)255; }
// the scratch's first bytes that must be zero before its first batch (later batches leave them zero)
inline size_t ro_zero_bytes(uint32_t T) { return 256 + ro_align(4ull * T); }
inline size_t ro_scratch_bytes(uint32_t n, uint32_t T)
{
    return ro_zero_bytes(T) + 2 * ro_align(4ull * T) + ro_align(8ull * kRoBucket * T) + ro_align(16ull * n) +
           ro_align(16ull * n) + ro_align(8ull * n) + ro_align(16ull * n) + ro_align(8ull * ((n + 63) / 64));
}
inline RoScratch ro_scratch_layout(void *base, uint32_t n, uint32_t T)
{
    uint8_t *b = static_cast<uint8_t *>(base);
    RoScratch s;
    s.ctr = reinterpret_cast<uint32_t *>(b);
    s.runCnt = reinterpret_cast<uint32_t *>(b + 256);
    b += ro_zero_bytes(T);
    s.runBase = reinterpret_cast<uint32_t *>(b);
    s.active = reinterpret_cast<uint32_t *>(b + ro_align(4ull * T));
    b += 2 * ro_align(4ull * T);
    s.bucket = reinterpret_cast<unsigned long long *>(b);
    b += ro_align(8ull * kRoBucket * T);
    s.recs = reinterpret_cast<RoRec *>(b);
    b += ro_align(16ull * n);
    s.runs = reinterpret_cast<RoRun *>(b);
    b += ro_align(16ull * n);
    s.placed = reinterpret_cast<unsigned long long *>(b);
    b += ro_align(8ull * n);
    s.sortTmp = reinterpret_cast<unsigned long long *>(b);
    b += ro_align(16ull * n);
    s.ovMask = reinterpret_cast<unsigned long long *>(b);
    return s;
}
hipError_t launch_ro_classify(const ReasDev &R, const uint8_t *pkts, uint32_t stride, const uint32_t *lens,
                              uint32_t n, uint64_t now, void *work, void *scratch, size_t scratchBytes,
                              hipStream_t stream);

// Gather copy of up to kCopySpansPerLaunch spans (passed by value in the kernel arguments).
constexpr uint32_t kCopySpansPerLaunch = 64;
struct CopySpan {
    uint64_t src, dst, bytes;
};
struct CopySpans {
    CopySpan s[kCopySpansPerLaunch];
    uint32_t n;
};
hipError_t launch_copy_spans(const CopySpans &cs, uint64_t largest, hipStream_t stream);

// d_count (optional): the event count is read on the device; nEvents is then its bound
hipError_t launch_segment(const e2sar_hip_seg_event *d_events, uint32_t nEvents,
                          uint32_t maxPacketsPerEvent, int lbVersion, uint32_t maxPld,
                          uint8_t *pkts, uint32_t stride, uint32_t *lens,
                          hipStream_t stream, const uint32_t *d_count = nullptr, const ReasDev *rec = nullptr,
                          bool dropCompleted = false);
hipError_t launch_relay_plan(const ReasDev &R, uint32_t first, uint32_t maxEvents, uint32_t maxPld,
                             uint64_t lbTick, uint32_t entropyBase, e2sar_hip_seg_event *d_events,
                             uint32_t *d_counts, hipStream_t stream);
hipError_t launch_reassemble(const ReasDev &R, const uint8_t *pkts, uint32_t stride,
                             const uint32_t *lens, uint32_t n, uint64_t now, hipStream_t stream);
// XCD-matched groups of a planned batch (seg_kernel's stripes) and the fused reassembly over them
uint32_t seg_groups(const e2sar_hip_seg_event *ev, uint32_t nEvents, uint32_t maxPacketsPerEvent, uint32_t maxPld,
                    uint32_t stride, uint32_t *starts, uint32_t cap);
hipError_t launch_reassemble_groups(const ReasDev &R, const uint8_t *pkts, uint32_t stride, const uint32_t *lens,
                                    uint32_t n, const uint32_t *starts, uint32_t nGroups, uint64_t now,
                                    hipStream_t stream);
// Chained form: segment each batch and reassemble the same datagrams, up to
// kChainMaxBatches batches in one launch (segreas_kernel).  Batch b: nEvents descriptors at
// events (pktBase from seg_plan), n datagrams into pkts/lens, tiles = n zeroed words (left
// zeroed by the launch); batches use distinct packet buffers.
constexpr uint32_t kChainMaxBatches = 8;
struct ChainBatch {
    const e2sar_hip_seg_event *events;
    uint8_t *pkts;
    uint32_t *lens;
    uint32_t *tiles;
    uint32_t nEvents, maxPacketsPerEvent, n;
    uint32_t start, nSeg, bpe, G;           // filled by launch_segreas
};
struct ChainBatches {
    ChainBatch b[kChainMaxBatches];
    uint32_t nb;
};
hipError_t launch_segreas(ChainBatches cb, int lbVersion, uint32_t maxPld, uint32_t stride, const ReasDev &R,
                          uint64_t now, hipStream_t stream);
hipError_t launch_reas_classify(const ReasDev &R, const uint8_t *pkts, uint32_t stride, const uint32_t *lens,
                                uint32_t n, uint64_t now, void *work, hipStream_t stream);
hipError_t launch_reas_scatter(const ReasDev &R, const uint8_t *pkts, uint32_t stride, uint32_t n,
                               const void *work, hipStream_t stream, bool nt);   // nt: streaming datagram loads
hipError_t launch_reas_scatter_classify(const ReasDev &R, uint32_t stride, const uint8_t *spk, uint32_t sn,
                                        const void *swork, const uint8_t *cpk, const uint32_t *clens, uint32_t cn,
                                        uint64_t now, void *cwork, hipStream_t stream, bool nt);
hipError_t launch_zero_words(void *p, uint64_t nWords, hipStream_t stream);   // p 4-byte aligned
hipError_t launch_fill_bytes(void *p, int value, uint64_t n, hipStream_t stream); // any alignment
hipError_t launch_gc(const ReasDev &R, uint64_t now, uint64_t timeout, hipStream_t stream);
hipError_t launch_recycle(const ReasDev &R, bool dropCompleted, hipStream_t stream);
// Move every in-progress event of `from` (slots + arena bytes) into the empty `to`
// table/arena (same ctl), then make `to`'s top and slot count current.
hipError_t launch_compact(const ReasDev &from, const ReasDev &to, hipStream_t stream);
size_t route_workspace_bytes(uint32_t n, uint32_t world);
// one launch: reserve per-workgroup room in each destination's region (atomicAdd on
// running[d]) and copy; datagrams past a region's cap are counted, not written
hipError_t launch_route_append(const uint8_t *pkts, uint32_t stride, const uint32_t *lens, uint32_t n, int withLB,
                               uint32_t world, uint32_t self, int excludeSelf, uint8_t *out, uint32_t *outLens,
                               uint32_t cap, uint32_t *running, hipStream_t stream);
hipError_t launch_route(const uint8_t *pkts, uint32_t stride, const uint32_t *lens, uint32_t n, int withLB,
                        uint32_t world, uint32_t self, int excludeSelf, uint8_t *out, uint32_t *outLens,
                        uint32_t *counts, void *workspace, hipStream_t stream, uint32_t cap = 0,
                        uint32_t *running = nullptr);   // cap > 0: append to per-rank regions of cap slots

}  // namespace e2sar_amd
