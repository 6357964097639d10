// sar_kernels.hip -- gfx950 kernels of the SAR data path.
//
//   seg_kernel      : event batch -> datagram batch   (replaces _send's fragment loop,
//                     e2sarDPSegmenter.cpp:702-770)
//   reas_classify   : datagram batch -> per-packet destination + event table updates
//                     (replaces the recv body's parse/validate/find-or-create/complete,
//                     e2sarDPReassembler.cpp:335-427)
//   reas_scatter    : payload bytes -> event buffers (the memcpy at cpp:391-392)
//   reas_gc         : timeout pass (cpp:252-274)
//
// All of it is byte movement bounded by HBM bandwidth; no MFMA.  The copy kernels move
// 16 bytes per lane per access: destination chunks are 16-byte aligned, and the source
// side is read with dword-aligned 16-byte loads (gfx950 serves dword-aligned
// global_load_dwordx4), so the 4-mod-16 skew that the 36-byte header puts between event
// bytes and datagram bytes costs no shuffles.
#include "sar_kernels.hpp"

#include "wire.hpp"

#include <algorithm>
#include <atomic>

namespace e2sar_amd {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(4))) u32x4_a4;   // 16-byte access at dword alignment

constexpr int kBlock = 256;
// Launch geometry, fixed at the measured best (DESIGN.md 4.5 holds every A/B behind these
// numbers; round 5 removed the build-time switches whose alternatives lost).
constexpr int kScatBlock = 256;             // scatter / pipelined scatter+classify workgroup
constexpr uint32_t kPollSleep = 1;          // s_sleep units (64 clocks) between table slot polls
constexpr int kReasU = 4;                   // 16-byte chunks per thread per copy round (fused kernel)
constexpr int kScatU = 4;                   // the same for the scatter forms
// ... and for slots above 4 KiB: one 8976-byte datagram (561 chunks) fills 73 % of a
// 768-chunk round instead of 55 % of 1024.  Config 3's split reassembly 210.6-212.7 ->
// 207.7-208.9 us (profiles/round5/xcd_order/ab.log; 8 chunks, two datagrams a round: 215 us)
constexpr int kScatUJumbo = 3;
constexpr int kScatBlockJumbo = 256;        // scatter workgroup size for slots above 4 KiB
// fused kernel: run tails of events of at least this many bytes add to the event
// accumulator after the copy, not during classification
constexpr uint32_t kDeferAccBytes = 4194304u;
// Split / pipelined scatter loads: non-temporal for datagrams that were written long before
// (not in the Infinity Cache), plain for a batch just written -- chosen per launch
// (launch_reas_scatter's nt; capi.cpp: E2SAR_HIP_REAS_COLD_DATAGRAMS, or a batch too large to
// be cached).  Cold: a 205 x 1 MiB batch's scatter 85.1 (nt) vs 89.3 us (plain); hot: 68.0
// (plain) vs 89.4 us (nt), reference-order batches 124.8 vs 148.1 us (profiles/round2/ab3/nt).
constexpr uint32_t kReasChunksPerBlock = 9216u;      // fused group budget before balancing

// Timeline trace (experiment builds only, -DE2SAR_TRACE=1): per workgroup, s_memrealtime
// (100 MHz) at start, after classification, after the barrier and at the end, plus HW_ID.
#ifndef E2SAR_TRACE
#define E2SAR_TRACE 0
#endif
#if E2SAR_TRACE
constexpr uint32_t kTraceBlocks = 16384;
__device__ uint64_t g_trace[3][kTraceBlocks * 4];
#define TRACE_AT(k, slot, i) \
    do { if (threadIdx.x == 0 && blockIdx.x < kTraceBlocks) g_trace[k][blockIdx.x * 4 + (slot)] = (i); } while (0)
// by the first active lane of wave 0 (inside divergent code)
#define TRACE_FIRST(k, slot, i) \
    do { if (threadIdx.x < 64 && blockIdx.x < kTraceBlocks && \
             threadIdx.x == (uint32_t)(__builtin_ffsll((long long)__ballot(1)) - 1)) \
             g_trace[k][blockIdx.x * 4 + (slot)] = (i); } while (0)
#define TRACE_WAIT() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#else
#define TRACE_AT(k, slot, i) do {} while (0)
#define TRACE_FIRST(k, slot, i) do {} while (0)
#define TRACE_WAIT() do {} while (0)
#endif
__device__ __forceinline__ uint64_t trace_now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ uint64_t trace_hwid()
{
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return ((uint64_t)x << 32) | v;
}

// Global-address-space accessors: the event/packet/arena pointers reach the kernels
// through descriptor tables, so without these hipcc falls back to flat_* accesses.
#define E2SAR_GLOBAL __attribute__((address_space(1)))
__device__ __forceinline__ u32x4 ld16(const uint8_t *p) { return *(const E2SAR_GLOBAL u32x4_a4 *)(p); }
__device__ __forceinline__ void st16(uint8_t *p, u32x4 v) { *(E2SAR_GLOBAL u32x4 *)(p) = v; }
__device__ __forceinline__ uint32_t ld4(const uint8_t *p) { return *(const E2SAR_GLOBAL uint32_t *)(p); }
__device__ __forceinline__ void st4(uint8_t *p, uint32_t v) { *(E2SAR_GLOBAL uint32_t *)(p) = v; }
__device__ __forceinline__ uint8_t ld1(const uint8_t *p) { return *(const E2SAR_GLOBAL uint8_t *)(p); }
// Non-temporal forms for bytes touched once: event bytes read by seg_kernel, event bytes
// written by reas_kernel.  Datagram bytes keep the default policy so a batch written by
// seg_kernel can still be in L2 / Infinity Cache when reas_kernel reads it.
__device__ __forceinline__ u32x4 ld16_nt(const uint8_t *p)
{
    return __builtin_nontemporal_load((const E2SAR_GLOBAL u32x4_a4 *)(p));
}
__device__ __forceinline__ void st16_nt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (E2SAR_GLOBAL u32x4 *)(p)); }
// 16-byte non-temporal store at a dword-aligned (not 16-byte-aligned) address: event
// bytes written by the reassembly kernels.  (Round 3, profiles/round3/ab_ntstore/ and
// s2_ab_store/: cache-allocating event stores evict the batch's datagrams from the Infinity
// Cache -- reas_kernel 74 -> 108 us; write-through (sc1) stores 153-220 us.)
__device__ __forceinline__ void st16u_nt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (E2SAR_GLOBAL u32x4_a4 *)(p)); }
__device__ __forceinline__ void st1(uint8_t *p, uint8_t v) { *(E2SAR_GLOBAL uint8_t *)(p) = v; }

// Agent-coherent (sc1) forms for bytes handed from one workgroup to another inside a
// launch (the chained segment -> reassemble form): the producer stores every handed-off
// byte write-through (sc1), waits for its stores, then signals with an agent-scope atomic;
// the consumer reads every handed-off byte with sc1 loads (MI355X_MICROARCH.md,
// inter-workgroup visibility, first hand-off row).  16-byte forms go through a buffer
// resource whose base is workgroup-uniform (an SGPR operand), with the per-lane offset in
// a VGPR.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void *base)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7FFFFFFF, 0x00020000);
}
constexpr int kCpolSc1 = 16;
__device__ __forceinline__ u32x4 ld16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, kCpolSc1);
}
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, kCpolSc1);
}
__device__ __forceinline__ uint32_t ld4_sc1(const uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st4_sc1(uint32_t *p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint8_t ld1_sc1(const uint8_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup barrier that orders LDS only.  __syncthreads() also waits for every global
// load and atomic the wave has outstanding; here a classifier's fire-and-forget counter
// atomics and the payload loads of the other waves stay in flight across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---------------------------------------------------------------------------------
// segmentation

__device__ __forceinline__ uint32_t low_bytes_mask(uint32_t n)   // keep the n (<4) low bytes
{
    return (n >= 4u) ? 0xFFFFFFFFu : ((1u << (8u * n)) - 1u);
}

// Payload dword at byte offset r (a multiple of 4) of a datagram payload of L bytes,
// zero past L.  Reads only the dword that holds byte r, never the next one.
__device__ __forceinline__ uint32_t pl_dword(const uint8_t *pl, uint32_t r, uint32_t L)
{
    if (r >= L) return 0u;
    const uint32_t w = ld4(pl + r);
    return (r + 4u > L) ? (w & low_bytes_mask(L - r)) : w;
}

// Header dword i (0..8) of the datagram; w5 (bufferOffset) is the only per-datagram word.
struct SegHdr {
    uint32_t w0, w1, w2, w3, w4, w6, w7, w8;
};

__device__ __forceinline__ uint32_t seg_hdr_byte(const SegHdr &h, uint32_t w5, uint32_t q)
{
    const uint32_t i = q >> 2;
    uint32_t w = h.w0;
    w = (i == 1) ? h.w1 : w;
    w = (i == 2) ? h.w2 : w;
    w = (i == 3) ? h.w3 : w;
    w = (i == 4) ? h.w4 : w;
    w = (i == 5) ? w5 : w;
    w = (i == 6) ? h.w6 : w;
    w = (i == 7) ? h.w7 : w;
    w = (i == 8) ? h.w8 : w;
    return (w >> (8u * (q & 3u))) & 0xFFu;
}

// Generic case (event not dword-aligned, or maxPldLen % 4 != 0): byte loads.
__device__ __forceinline__ u32x4 seg_chunk_bytes(const SegHdr &h, uint32_t w5, const uint8_t *pl,
                                                 uint32_t L, uint32_t c)
{
    uint32_t o[4];
#pragma unroll
    for (uint32_t d = 0; d < 4; d++) {
        uint32_t w = 0;
#pragma unroll
        for (uint32_t b = 0; b < 4; b++) {
            const uint32_t q = 16u * c + 4u * d + b;
            uint32_t byte = 0;
            if (q < kLBREHdrLen) byte = seg_hdr_byte(h, w5, q);
            else if (q - kLBREHdrLen < L) byte = ld1(pl + (q - kLBREHdrLen));
            w |= byte << (8u * b);
        }
        o[d] = w;
    }
    u32x4 v;
    v.x = o[0];
    v.y = o[1];
    v.z = o[2];
    v.w = o[3];
    return v;
}

// Drop the s (0..3, lane-varying) lowest dwords of x, shifting the rest down, zero fill.
__device__ __forceinline__ u32x4 rot_down(u32x4 x, uint32_t s)
{
    u32x4 o;
    o.x = (s == 0u) ? x.x : (s == 1u) ? x.y : (s == 2u) ? x.z : x.w;
    o.y = (s == 0u) ? x.y : (s == 1u) ? x.z : (s == 2u) ? x.w : 0u;
    o.z = (s == 0u) ? x.z : (s == 1u) ? x.w : 0u;
    o.w = (s == 0u) ? x.w : 0u;
    return o;
}

// Zero the bytes of o at and past n (n in [0, 16]).
__device__ __forceinline__ u32x4 keep_low_bytes(u32x4 o, uint32_t n)
{
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const int vb = (int)n - 4 * d;
        o[d] = (vb <= 0) ? 0u : (vb < 4) ? (o[d] & low_bytes_mask((uint32_t)vb)) : o[d];
    }
    return o;
}

// grid.x = nEvents * blocksPerEvent; each block owns kBlock*U consecutive 16-byte
// chunks of ONE event's datagram range (event-major: every event field is a scalar).
// Datagram k of the event sits at pkts + (pktBase + k) * stride, so chunk j of the
// event lands at pkts + pktBase*stride + 16*j: the stores of a block are one contiguous
// run of memory.
//
// Chunk c of a datagram with payload pl[0, L): c = 0, 1 are LB / RE header words, c = 2
// is the RE eventNum low word + payload 0..11, c >= 3 is payload [16c-36, 16c-20).
// Every lane issues exactly one unconditional 16-byte load per chunk (phase 1) -- the
// window is slid back so it never leaves the event (a tail chunk reads the 16 bytes
// that END at its last dword, then shifts them down in registers) -- and only phase 2
// consumes them.  So no load result sits behind a branch and all U loads of a lane are
// in flight together.
// dCount (optional): the number of events is read on the device (the relay form, whose
// event table is built by relay_plan_kernel); blocks of events past it exit.
// The dword fast path (16-byte loads at dword alignment) is chosen per event from the
// event's own address and maxPld: a block handles one event, so the choice is uniform.
//
// HO (the chained form, segreas_kernel): every datagram byte and length is stored sc1 and,
// once the block's stores are done, the block adds the number of index-space chunks it
// covered in each reassembly group's range of datagrams to that group's counter
// (tiles[slot / tileG]); a group starts when its counter reaches its slots x stride/16.
constexpr int kSegBlock = 256;       // seg_kernel threads per workgroup (128 / 512 lost)
// seg_kernel<4> (16-KiB workgroups, events of more than 4 MiB of datagrams) at most 6
// workgroups per CU: config 3's segmentation 180.0-181.4 vs 185.3 us; seg_kernel<2> loses
// with any cap (7 / 6 / 5 per CU: 67.4-68.2 / 71.3-72.3 / 76.6-77.9 vs 67.7-70.0 us at 1 MiB;
// profiles/round4/ab/seg_occupancy.log)
constexpr uint32_t kSeg4PerCU = 6;
// One round of a segmentation block: index-space chunks [j0, j0 + SB*U) of event ev,
// bounded by jEnd (the event's chunk count, or the end of a local chained range).
struct SegEv {
    SegHdr h;
    const uint8_t *data;
    uint32_t pktBase, bytes, npk, spc, maxPld;
    float rspc;
    bool A4;
};

__device__ __forceinline__ SegEv seg_ev(const e2sar_hip_seg_event &ev, int lbVersion, uint32_t maxPld, uint32_t stride)
{
    HdrWords hw;
    lbre_words(hw, lbVersion, ev.entropy, ev.lbTick, ev.dataId, 0u, ev.bytes, ev.eventNum);
    SegEv E;
    E.h = SegHdr{hw.w[0], hw.w[1], hw.w[2], hw.w[3], hw.w[4], hw.w[6], hw.w[7], hw.w[8]};
    E.data = ev.data;
    E.pktBase = ev.pktBase;
    E.bytes = ev.bytes;
    E.npk = (ev.bytes + maxPld - 1u) / maxPld;
    E.spc = stride >> 4;
    E.maxPld = maxPld;
    E.rspc = 1.0f / (float)E.spc;
    E.A4 = (((uintptr_t)ev.data | maxPld) & 3u) == 0u;
    return E;
}

template <int U, bool HO, int SB>
__device__ __forceinline__ void seg_round(const SegEv &E, uint8_t *__restrict__ out, __amdgpu_buffer_rsrc_t outR,
                                          uint32_t outJ0, const uint8_t *safe, uint32_t *__restrict__ lens,
                                          uint32_t j0, uint32_t jEnd)
{
    const SegHdr h = E.h;        // a copy: a reference into E leaves E in scratch memory
    const uint32_t bytes = E.bytes, npk = E.npk, spc = E.spc, maxPld = E.maxPld;
    const bool A4 = E.A4;
    const float rspc = E.rspc;
    u32x4 x[U];
    uint32_t jj[U], cc[U], LL[U], kk[U], sh[U];
    bool rare[U];
    // ---- phase 1: one load per chunk ----
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t j = j0 + (uint32_t)u * SB + threadIdx.x;
        jj[u] = 0xFFFFFFFFu;
        cc[u] = LL[u] = kk[u] = sh[u] = 0;
        rare[u] = false;
        const uint8_t *a = safe;
        if (j < jEnd) {
            // k = j / spc: a float reciprocal and a +-1 correction while k < 2^22 (the
            // estimate is then off by less than one); integer division for the datagrams of
            // larger events (npk is event-uniform, so the branch never diverges)
            uint32_t k;
            if (npk < (1u << 22)) {
                k = (uint32_t)((float)j * rspc);
                if (k * spc > j) k--;
                else if ((k + 1u) * spc <= j) k++;
            } else {
                k = j / spc;
            }
            const uint32_t c = j - k * spc;
            const uint32_t off = k * maxPld;
            const uint32_t L = (bytes - off > maxPld) ? maxPld : bytes - off;
            if (c == 0u && lens) {
                if (HO) st4_sc1(lens + E.pktBase + k, kLBREHdrLen + L);
                else lens[E.pktBase + k] = kLBREHdrLen + L;
            }
            if (16u * c < kLBREHdrLen + L) {          // else: chunk wholly past the datagram end
                jj[u] = j;
                cc[u] = c;
                LL[u] = L;
                kk[u] = k;
                const uint8_t *pl = E.data + off;
                if (!A4) {
                    rare[u] = true;
                } else if (c >= 3u) {
                    const uint32_t r = 16u * c - kLBREHdrLen;
                    const uint32_t n = (L - r < 16u) ? L - r : 16u;
                    const uint32_t rn = (n + 3u) & ~3u;
                    sh[u] = (16u - rn) >> 2;
                    a = pl + (r + rn - 16u);
                } else if (c == 2u) {
                    if (k > 0u && L >= 12u) a = pl - 4;       // previous datagram's last payload dword
                    else rare[u] = true;                      // event start / tiny datagram
                }
            }
        }
        x[u] = ld16_nt(a);
    }
    // ---- phase 2: header words, shifts, tail masks, stores ----
#pragma unroll
    for (int u = 0; u < U; u++) {
        if (jj[u] == 0xFFFFFFFFu) continue;
        const uint32_t c = cc[u], L = LL[u];
        const uint32_t w5 = bswap32(kk[u] * maxPld);
        const uint8_t *pl = E.data + kk[u] * maxPld;
        u32x4 o;
        if (rare[u]) {
            if (!A4) {
                o = seg_chunk_bytes(h, w5, pl, L, c);
            } else {        // c == 2 at an event start or in a datagram of < 12 payload bytes
                o.x = h.w8;
                o.y = pl_dword(pl, 0u, L);
                o.z = pl_dword(pl, 4u, L);
                o.w = pl_dword(pl, 8u, L);
            }
        } else if (c >= 3u) {
            const uint32_t r = 16u * c - kLBREHdrLen;
            o = rot_down(x[u], sh[u]);
            if (L - r < 16u) o = keep_low_bytes(o, L - r);
        } else if (c == 2u) {
            o = x[u];
            o.x = h.w8;
        } else if (c == 1u) {
            o = u32x4{h.w4, w5, h.w6, h.w7};
        } else {
            o = u32x4{h.w0, h.w1, h.w2, h.w3};
        }
        // plain stores: the batch stays in the Infinity Cache for the reassembly that reads it
        // next (nt stores: reas_kernel 97.8 vs 74 us, round 3)
        if (HO) st16_sc1(outR, 16u * (jj[u] - outJ0), o);
        else st16(out + 16u * jj[u], o);
    }
}

template <int U, bool HO, int SB = kBlock>
__device__ __forceinline__ void seg_block(const e2sar_hip_seg_event *__restrict__ events, uint32_t blocksPerEvent,
                                          int lbVersion, uint32_t maxPld, uint8_t *__restrict__ pkts, uint32_t stride,
                                          uint32_t *__restrict__ lens, const uint32_t *__restrict__ dCount,
                                          uint32_t blk, uint32_t tileG, uint32_t *__restrict__ tiles)
{
    TRACE_AT(1, 0, trace_now());
    const uint32_t e = blk / blocksPerEvent;
    const uint32_t bx = blk - e * blocksPerEvent;
    if (dCount && e >= *dCount) return;
    const e2sar_hip_seg_event ev = events[e];
    const SegEv E = seg_ev(ev, lbVersion, maxPld, stride);
    const uint32_t spc = E.spc;
    const uint32_t nch = E.npk * spc;
    const uint32_t j0 = bx * (uint32_t)(SB * U);
    if (j0 >= nch) return;

    uint8_t *const out = pkts + (uint64_t)ev.pktBase * stride;
    const __amdgpu_buffer_rsrc_t outR = brsrc(out + 16ull * j0);        // HO stores only
    const uint8_t *const safe = reinterpret_cast<const uint8_t *>(events + e);   // >= 16 valid bytes
    seg_round<U, HO, SB>(E, out, outR, j0, safe, lens, j0, nch);
    if (HO) {
        // every storing wave waits for its write-through stores, then one wave signals for
        // the workgroup behind the barrier
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x < 64) {
            const uint32_t j1 = (j0 + (uint32_t)(SB * U) < nch) ? j0 + (uint32_t)(SB * U) : nch;
            const uint64_t s0 = (uint64_t)ev.pktBase + j0 / spc, s1 = (uint64_t)ev.pktBase + (j1 - 1u) / spc;
            const uint64_t t0 = s0 / tileG, t1 = s1 / tileG;
            for (uint64_t t = t0 + (threadIdx.x & 63u); t <= t1; t += 64u) {
                const uint64_t tlo = t * tileG, thi = tlo + tileG;        // slots of group t
                const uint64_t clo = (tlo > ev.pktBase) ? (tlo - ev.pktBase) * spc : 0u;
                const uint64_t chi = (thi - ev.pktBase) * spc;            // thi > s0 >= pktBase
                const uint64_t lo = clo > j0 ? clo : j0, hi = chi < j1 ? chi : j1;
                __hip_atomic_fetch_add(tiles + t, (uint32_t)(hi - lo), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
#if E2SAR_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    TRACE_AT(1, 2, trace_hwid());
    TRACE_AT(1, 3, trace_now());
#endif
}

// stripe > 0 (XCD stripes): the dispatcher hands workgroup b to XCD b mod 8 (round robin,
// checked by tools/ubench_l2keep.hip), and workgroup b = 8k + x takes unit
// ((k / stripe) * 8 + x) * stripe + k % stripe, so units [m * stripe, (m + 1) * stripe) --
// a stripe of consecutive datagrams -- are all written on XCD m mod 8.  A reassembly
// launched with the matching group table (seg_groups) then reads every stripe on the XCD
// that wrote it, which reads measurably faster than lines another XCD wrote, also from
// the Infinity Cache.  Units are numbered e * blocksPerEvent + bx as
// without stripes; units past nUnits exit.
__device__ void recycle_slots(const ReasDev &R, uint32_t s, int dropCompleted);

// recMode != 0 (e2sar_hip_segment_batch_recycle): workgroups from nSegBlocks on recycle the
// reassembler `rec` (reas_recycle_kernel's work; 2 = also drop completed records) instead of
// segmenting.  They run at the end of the launch, in the slots the last seg blocks free; no
// seg block touches the table, and the reassembly that used it ran before this launch.
template <int U>
__global__ __launch_bounds__(kSegBlock) void seg_kernel(const e2sar_hip_seg_event *__restrict__ events,
                                                              uint32_t blocksPerEvent, int lbVersion,
                                                              uint32_t maxPld, uint8_t *__restrict__ pkts,
                                                              uint32_t stride, uint32_t *__restrict__ lens,
                                                              const uint32_t *__restrict__ dCount, uint32_t stripe,
                                                              uint32_t nUnits, ReasDev rec, uint32_t nSegBlocks,
                                                              int recMode)
{
    uint32_t blk = blockIdx.x;
    if (recMode && blk >= nSegBlocks) {
        recycle_slots(rec, (blk - nSegBlocks) * kSegBlock + threadIdx.x, recMode == 2);
        return;
    }
    if (stripe) {
        const uint32_t x = blk & 7u, k = blk >> 3;
        blk = ((k / stripe) * 8u + x) * stripe + k % stripe;
        if (blk >= nUnits) return;
    }
    seg_block<U, false, kSegBlock>(events, blocksPerEvent, lbVersion, maxPld, pkts, stride, lens, dCount,
                                         blk, 1u, nullptr);
}

// ---------------------------------------------------------------------------------
// reassembly: event table protocol
//
// slot.state: EMPTY -> BUSY (CAS by the inserting lane) -> READY (published with the key)
// -> DONE (completed) / LOST (GC'd).  A lookup claims first: CAS EMPTY->BUSY either makes
// the lane the creator (one round trip) or returns the slot's state.  The creator takes its
// buffer from the arena and publishes record B {bufOff, bytes, bvalid=1} and record A
// {READY, dataId, eventNum} as two 16-byte agent-scope (sc1) stores, without waiting for
// them; other lanes read A and B together (two sc1 loads, one round trip) until A is READY
// and B valid.  acc starts at 0 because a slot is EMPTY only after it was zeroed (slots
// are never reused within an arena epoch).

enum : uint32_t { kEmpty = 0, kBusy = 1, kReady = 2, kDone = 3, kLost = 4 };

template <typename T>
__device__ __forceinline__ T ld_agent(const T *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
struct id_t_ { typedef T type; };
template <typename T>
__device__ __forceinline__ void st_agent(T *p, typename id_t_<T>::type v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// occupancy shard of a table slot (ReasOcc follows the ReasShard array)
__device__ __forceinline__ unsigned long long *occ_in_progress(const ReasDev &R, uint32_t slot)
{
    return reinterpret_cast<unsigned long long *>(&(reinterpret_cast<ReasOcc *>(R.shards + kShards) + slot % kShards)->inProgress);
}
__device__ __forceinline__ unsigned long long *occ_table_used(const ReasDev &R, uint32_t slot)
{
    return reinterpret_cast<unsigned long long *>(&(reinterpret_cast<ReasOcc *>(R.shards + kShards) + slot % kShards)->tableUsed);
}
// 16-byte agent-scope store and the pair of 16-byte agent-scope loads of records A and B
// (the forms the compiler emits for 4/8-byte agent-scope atomics, at 16 bytes).  The
// loads wait for their own results inside the asm.
__device__ __forceinline__ void st16_agent(void *p, u32x4 v)
{
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void ld_slot_ab(const ReasSlot *sl, u32x4 &A, u32x4 &B)
{
    asm volatile("global_load_dwordx4 %0, %2, off sc1\n\t"
                 "global_load_dwordx4 %1, %2, off offset:16 sc1\n\t"
                 "s_waitcnt vmcnt(0)"
                 : "=&v"(A), "=&v"(B)
                 : "v"(sl)
                 : "memory");
}

__device__ __forceinline__ uint32_t slot_hash(uint64_t ev, uint32_t d, uint32_t mask)
{
    // pair_hash (e2sarUtil.hpp:526-533) then a 64-bit finaliser so that event numbers
    // that differ only in high bits (ticks) or in dataId spread over the table.
    uint64_t t = d;
    uint64_t h = ev ^ (t | t << 16 | t << 32 | t << 48);
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    return (uint32_t)h & mask;
}

struct LookupResult {
    uint32_t slot;      // kNoSlot on failure
    uint32_t bytes;     // slot's bufferLength (from the packet that created it)
    uint64_t bufOff;    // arena offset or kNoBuf
};
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
constexpr uint64_t kNoBuf = ~0ull;
constexpr uint32_t kSpinLimit = 1u << 22;

// Record B's bvalid in reference-order mode for a key registered by ro_key_kernel whose
// event item (buffer, counters) does not exist yet: ro_walk_kernel creates items.
constexpr uint32_t kBNoItem = 2u;

// Called by a whole wave: lanes with want == false only take part in the loop.  The wave
// loops until every wanting lane has a result, and every pass is straight-line (claim;
// creators publish; the others read), so a lane never waits inside a divergent branch
// for a slot that another lane of the same wave is still creating.
// keyOnly (reference-order mode): a creator registers the key without an event buffer
// (record B = {kNoBuf, 0, kBNoItem}); the walk that follows creates the items.
template <bool keyOnly = false>
__device__ LookupResult find_or_create(const ReasDev &R, bool want, uint64_t ev, uint32_t d, uint32_t blen,
                                       uint64_t now)
{
    LookupResult res{kNoSlot, 0, kNoBuf};
    const uint32_t mask = R.tableSlots - 1u;
    uint32_t h = slot_hash(ev, d, mask);
    uint32_t probes = 0, spins = 0;
    bool active = want;
#if E2SAR_TRACE
    uint32_t pass = 0;
#endif
    bool claimed = false;          // the current slot is known to be past EMPTY: poll by loads
    while (__ballot(active)) {
        bool waiting = false, advance = false;
        if (active) {
            ReasSlot *sl = R.slots + h;
            // a slot never returns to EMPTY within an arena epoch, so once a claim has
            // failed, later passes poll records A/B with loads instead of repeating the CAS
            // (A/B: +1.1 % at 1 MiB / MTU 1500, +1.8 % at 8 MiB / MTU 9000)
            const uint32_t old = claimed ? (uint32_t)kBusy : atomicCAS(&sl->state, (uint32_t)kEmpty, (uint32_t)kBusy);
#if E2SAR_TRACE
            if (pass == 0) {
                TRACE_WAIT();
                TRACE_FIRST(2, 1, trace_now());
            }
#endif
            if (old == kEmpty && keyOnly) {
                st16_agent(&sl->bufOff, u32x4{(uint32_t)kNoBuf, (uint32_t)(kNoBuf >> 32), 0u, kBNoItem});
                st16_agent(sl, u32x4{(uint32_t)kReady, d, (uint32_t)ev, (uint32_t)(ev >> 32)});
                atomicAdd(occ_table_used(R, h), 1ull);
                res.slot = h;
                active = false;
            } else if (old == kEmpty) {
                // this lane owns the slot: buffer, then records B and A
                const uint64_t need = ((uint64_t)blen + 255ull) & ~255ull;
                uint64_t boff = atomicAdd(&R.ctl->arenaTop, (unsigned long long)(need ? need : 256ull));
                if (boff + blen > R.arenaBytes) {
                    boff = kNoBuf;
                    atomicOr(&R.ctl->errorFlags, 2u);
                }
                st_agent(&sl->created, now);
                st16_agent(&sl->bufOff, u32x4{(uint32_t)boff, (uint32_t)(boff >> 32), blen, 1u});
                st16_agent(sl, u32x4{(uint32_t)kReady, d, (uint32_t)ev, (uint32_t)(ev >> 32)});
                atomicAdd(occ_in_progress(R, h), 1ull);
                atomicAdd(occ_table_used(R, h), 1ull);
                res.slot = h;
                res.bytes = blen;
                res.bufOff = boff;
                active = false;
            } else if (old == kBusy || old == kReady) {
                u32x4 A, B;
                ld_slot_ab(sl, A, B);
                if (A.x == kReady && B.w != 0u) {
                    if (A.y == d && (((uint64_t)A.w << 32) | A.z) == ev) {
                        res.slot = h;
                        res.bytes = B.z;
                        res.bufOff = ((uint64_t)B.y << 32) | B.x;
                        active = false;
                    } else {
                        advance = true;                                // another event's slot
                    }
                } else if (A.x == kDone || A.x == kLost) {
                    advance = true;                                    // DONE / LOST meanwhile
                } else {
                    waiting = true;                // not published yet, or a read that overtook the claim
                    claimed = true;
                }
            } else {
                advance = true;                                        // DONE / LOST
            }
            if (advance) {
                claimed = false;
                h = (h + 1u) & mask;
                if (++probes >= R.tableSlots) {
                    atomicOr(&R.ctl->errorFlags, 1u);
                    active = false;
                }
            }
            if (waiting && ++spins > kSpinLimit) {
                atomicOr(&R.ctl->errorFlags, 4u);
                active = false;
            }
        }
        if (__ballot(waiting)) __builtin_amdgcn_s_sleep(kPollSleep);
#if E2SAR_TRACE
        pass++;
#endif
    }
#if E2SAR_TRACE
    if (__ballot(want)) {
        TRACE_FIRST(2, 2, trace_now());
        TRACE_FIRST(2, 3, pass);
    }
#endif
    return res;
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src)
{
    const uint32_t lo = __shfl((uint32_t)v, src);
    const uint32_t hi = __shfl((uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
// DPP forms of the wave's neighbour moves and its prefix sum: VALU instructions instead of
// ds_bpermute round trips through the LDS pipe (the classification runs ~30 of those in a
// dependent chain otherwise, ~1 us at kernel start).  Whole wave active.
__device__ __forceinline__ uint32_t lane_prev(uint32_t v, uint32_t fill)     // lane i <- lane i-1
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x138 /* wave_shr:1 */, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t lane_next(uint32_t v, uint32_t fill)     // lane i <- lane i+1
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x130 /* wave_shl:1 */, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111 /* row_shr:1 */, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112 /* row_shr:2 */, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114 /* row_shr:4 */, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118 /* row_shr:8 */, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142 /* row_bcast:15 */, 0xa, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143 /* row_bcast:31 */, 0xc, 0xf, false);
    return v;
}

// Raw header words of one datagram, loaded before the payload loads of the block so the
// classification chain overlaps them.
struct RawHdr {
    uint32_t len;
    u32x4 re;        // RE header dwords 0..3
    uint32_t re4;    // RE header dword 4 (eventNum low word)
};

template <bool HO = false>
__device__ __forceinline__ RawHdr load_hdr(const ReasDev &R, const uint8_t *__restrict__ pkts, uint32_t stride,
                                           const uint32_t *__restrict__ lens, uint32_t p)
{
    const uint8_t *re = pkts + (uint64_t)p * stride + (R.withLB ? kLBHdrLen : 0u);   // 16-byte aligned
    RawHdr h;
    if (HO) {       // bytes handed off inside the launch (chained form): sc1 loads
        h.len = ld4_sc1(lens + p);
        h.re.x = ld4_sc1(reinterpret_cast<const uint32_t *>(re));
        h.re.y = ld4_sc1(reinterpret_cast<const uint32_t *>(re + 4));
        h.re.z = ld4_sc1(reinterpret_cast<const uint32_t *>(re + 8));
        h.re.w = ld4_sc1(reinterpret_cast<const uint32_t *>(re + 12));
        h.re4 = ld4_sc1(reinterpret_cast<const uint32_t *>(re + 16));
        return h;
    }
    h.len = lens[p];
    h.re = ld16(re);
    h.re4 = ld4(re + 16);
    return h;
}

// True for an event another rank owns (ReasDev.ownWorld > 1; owner = eventNum % world, the
// key e2sarDPReassembler.hpp:224-229 steers receive threads by).  The modulo runs only when
// ownership is set (a uniform branch).
__device__ __forceinline__ bool foreign_event(const ReasDev &R, uint64_t ev)
{
    return R.ownWorld > 1u && (uint32_t)(ev % R.ownWorld) != R.ownSelf;
}

// Per-packet counters of one wave (cpp:331-357): one atomic per wave per counter, sharded.
// Whole wave active.
__device__ __forceinline__ void wave_stats(const ReasDev &R, bool live, uint32_t len, bool bad, bool derr,
                                           uint32_t shard)
{
    const uint64_t np = __builtin_popcountll(__ballot(live));
    const uint64_t nbad = __builtin_popcountll(__ballot(bad));
    const uint64_t nder = __builtin_popcountll(__ballot(derr));
    // 64 lengths summed as 16-bit halves (each half-sum fits 32 bits, whatever the lengths)
    const uint32_t tl = live ? len : 0u;
    const uint64_t tb = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(tl & 0xFFFFu), 63) +
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(tl >> 16), 63) << 16);
    if ((threadIdx.x & 63u) == 0) {
        ReasShard *sh = R.shards + (shard % kShards);
        if (np) atomicAdd(&sh->totalPackets, (unsigned long long)np);
        if (tb) atomicAdd(&sh->totalBytes, (unsigned long long)tb);
        if (nbad) atomicAdd(&sh->badHeaderDiscards, (unsigned long long)nbad);
        if (nder) atomicAdd(&sh->dataErrCnt, (unsigned long long)nder);
    }
}

// RE header of one datagram -> key, offset, event length, payload length (cpp:340-357;
// REHdr::validate, e2sarHeaders.hpp:98-101).  Datagrams too short for the headers are bad
// headers; one longer than its slot (a truncated receive) is a data error.
struct ParsedHdr {
    uint64_t ev;
    uint32_t d, off, blen, pl;
    bool ok, bad, derr;
};
__device__ __forceinline__ ParsedHdr parse_hdr(const RawHdr &raw, uint32_t hl, uint32_t stride, bool live)
{
    ParsedHdr h{0, 0, 0, 0, 0, false, false, false};
    if (!live) return h;
    if (raw.len < hl) {
        h.bad = true;
    } else if (raw.len > stride) {
        h.derr = true;
    } else if (!re_valid(raw.re.x)) {
        h.bad = true;
    } else {
        h.d = bswap16(raw.re.x >> 16);
        h.off = bswap32(raw.re.y);
        h.blen = bswap32(raw.re.z);
        h.ev = ((uint64_t)bswap32(raw.re.w) << 32) | bswap32(raw.re4);
        h.pl = raw.len - hl;
        h.ok = true;
    }
    return h;
}

// Per-lane classification result; the run tail's counter update is issued during
// classification and its return value consumed only after the payload stores.
struct Classified {
    PktInfo info;
    uint64_t ev;
    uint64_t boff;
    unsigned long long old;   // value returned by the run tail's atomic add
    uint32_t d, slot, sbytes, rb, rc;
    bool tailAdd;
};

// Executed by one whole wave (all 64 lanes, any subset live).  Consecutive lanes that
// carry the same (eventNum, dataId) form a run: only the run head touches the event
// table and only the run tail adds to the event's byte/fragment counter, so the
// per-event atomics are per run, not per datagram.
// DeferAcc: the run tail's add to the event's accumulator is left to the caller (the fused
// kernel issues it after its copy, so the copy's waits never sit behind that atomic).
template <bool DeferAcc = false>
__device__ Classified classify_wave(const ReasDev &R, const RawHdr &raw, uint32_t stride, bool live,
                                    uint64_t now, uint32_t shard)
{
    const int lane = threadIdx.x & 63;
    const uint32_t hl = R.withLB ? kLBREHdrLen : kREHdrLen;

    uint32_t len = live ? raw.len : 0u;
    bool ok = false, bad = false, derr = false;
    uint64_t ev = 0;
    uint32_t d = 0, off = 0, blen = 0, pl = 0;
    if (live) {
        if (len < hl) {
            bad = true;                                       // too short to hold the headers
        } else if (len > stride) {
            derr = true;                                      // datagram overruns its slot
        } else if (!re_valid(raw.re.x)) {
            bad = true;                                       // cpp:351-357
        } else {
            d = bswap16(raw.re.x >> 16);
            off = bswap32(raw.re.y);
            blen = bswap32(raw.re.z);
            ev = ((uint64_t)bswap32(raw.re.w) << 32) | bswap32(raw.re4);
            pl = len - hl;
            ok = true;
        }
    }
    if (ok && foreign_event(R, ev)) {                         // another rank's event: not ours
        live = false;
        ok = false;
        len = 0;
        ev = 0;
        d = off = blen = pl = 0;
    }

    // ---- runs of equal keys ----
    const uint64_t pev = ((uint64_t)lane_prev((uint32_t)(ev >> 32), 0u) << 32) | lane_prev((uint32_t)ev, 0u);
    const uint64_t nev = ((uint64_t)lane_next((uint32_t)(ev >> 32), 0u) << 32) | lane_next((uint32_t)ev, 0u);
    const uint32_t pd = lane_prev(d, 0u), nd = lane_next(d, 0u);
    const uint32_t pok = lane_prev(ok ? 1u : 0u, 0u), nok = lane_next(ok ? 1u : 0u, 0u);
    const bool head = ok && (lane == 0 || !pok || pev != ev || pd != d);
    const bool tail = ok && (lane == 63 || !nok || nev != ev || nd != d);

    // (Round 3 tried a group-key pre-pass -- the first and last key of every fused group
    // resolved by a kernel of its own -- and removed it: -1 us in reas_kernel, +9 us of
    // pre-pass)
    const LookupResult lr = find_or_create(R, head, ev, d, blen, now);

    const uint64_t H = __ballot(head);
    const uint64_t le = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
    const uint64_t hm = H & le;
    const int myhead = hm ? 63 - __builtin_clzll(hm) : lane;
    const uint32_t slot = __shfl(lr.slot, myhead);
    const uint32_t sbytes = __shfl(lr.bytes, myhead);
    const uint64_t boff = shfl_u64(lr.bufOff, myhead);

    // bounds against the event's length (the reference memcpy has no check, cpp:391)
    bool take = ok && slot != kNoSlot;
    if (take && (uint64_t)off + pl > sbytes) {
        take = false;
        derr = true;
    }
    // segmented sums over the run (inclusive scans, then difference at the head)
    const uint32_t xb = take ? pl : 0u, xc = take ? 1u : 0u;
    const uint32_t ib = wave_incl_scan(xb), ic = wave_incl_scan(xc);
    const uint32_t hb = __shfl(ib - xb, myhead), hc = __shfl(ic - xc, myhead);

    Classified out;
    out.ev = ev;
    out.d = d;
    out.slot = slot;
    out.sbytes = sbytes;
    out.boff = boff;
    out.rb = ib - hb;
    out.rc = ic - hc;
    out.old = 0;
    out.tailAdd = tail && slot != kNoSlot;
    if (out.tailAdd && !(DeferAcc && sbytes >= kDeferAccBytes)) {
        const uint64_t add = ((uint64_t)out.rc << kAccFragShift) | out.rb;
        out.old = atomicAdd(&R.slots[slot].acc, (unsigned long long)add);   // consumed in classify_finish
    }

    const bool scatter = take && boff != kNoBuf;
    out.info.dst = scatter ? (uint64_t)(R.arena + boff + off) : 0ull;
    out.info.plen = scatter ? pl : 0u;
    out.info.hl = hl;
    if (ok && slot == kNoSlot) derr = true;                    // table full / probe timeout

    wave_stats(R, live, len, bad, derr, shard);
    return out;
}

// Completion (cpp:403-427): erase from the table, count, and hand the event to the
// completed queue (or record it lost when the queue is full or it had no buffer).
// keepSlot (reference-order mode): the walk that found the completion already left the
// slot in its final state (a later fragment of the key may have started a new item).
__device__ void complete_event(const ReasDev &R, uint32_t slot, uint64_t ev, uint64_t boff, uint32_t bytes,
                               uint32_t d, uint32_t frags, bool keepSlot = false)
{
    ReasSlot *sl = R.slots + slot;
    if (!keepSlot) st_agent(&sl->state, (uint32_t)kDone);      // erase from the map (cpp:409)
    atomicAdd(&R.shards[slot % kShards].eventSuccess, 1ull);   // cpp:426
    atomicAdd(occ_in_progress(R, slot), ~0ull);
    bool lostOnEnqueue = (boff == kNoBuf);
    if (!lostOnEnqueue) {
        const uint32_t idx = atomicAdd(&R.ctl->nCompleted, 1u);
        if (idx < R.queueCapacity) {
            e2sar_hip_event_rec rec;
            rec.eventNum = ev;
            rec.arenaOffset = boff;
            rec.bytes = bytes;
            rec.dataId = (uint16_t)d;
            rec.flags = 0;
            rec.numFragments = frags;
            rec.reserved = 0;
            R.completed[idx] = rec;
        } else {
            lostOnEnqueue = true;                              // queue full (hpp:140-145)
        }
    }
    if (lostOnEnqueue) {
        atomicAdd(&R.ctl->enqueueLoss, 1ull);
        const uint32_t li = atomicAdd(&R.ctl->nLost, 1u);
        if (li < R.lostCapacity) {
            e2sar_hip_lost_rec lr;
            lr.eventNum = ev;
            lr.numFragments = frags;
            lr.dataId = (uint16_t)d;
            lr.enqueueLoss = 1;
            lr.reserved = 0;
            R.lost[li] = lr;
        }
    }
}

// True when this run tail's add brought curBytes to the event length (cpp:403).
__device__ __forceinline__ bool completes(const Classified &c)
{
    if (!c.tailAdd) return false;
    const uint64_t nb = (c.old & kAccBytesMask) + c.rb;
    return c.rc > 0 && nb == c.sbytes;
}

__device__ __forceinline__ void classify_finish(const ReasDev &R, const Classified &c)
{
    if (!completes(c)) return;
    complete_event(R, c.slot, c.ev, c.boff, c.sbytes, c.d, (uint32_t)(c.old >> kAccFragShift) + c.rc);
}

// ---------------------------------------------------------------------------------
// reassembly: one fused kernel

// Dwords [lo/4, hi/4) of the register chunk v (lo < hi, both multiples of 4) to dst + lo:
// a payload's first and last 16-byte chunk.  The store instructions a wave issues are what
// its lanes need between them (exec-masked), so a wave holding one edge lane pays every
// form the edge takes: one store of the edge's length (dword, dwordx2 or dwordx3).  (Round
// 3, profiles/round3/s3_edge/: four conditional dword stores per edge -- four store
// instructions per edge wave -- were slower: config 3 scatter 227.6-232.0 vs 225.7-227.7 us.)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef u32x2 __attribute__((aligned(4))) u32x2_a4;
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
__device__ __forceinline__ void st8(uint8_t *p, uint32_t a, uint32_t b)
{
    *(E2SAR_GLOBAL u32x2_a4 *)(p) = u32x2{a, b};
}
__device__ __forceinline__ void st12(uint8_t *p, uint32_t a, uint32_t b, uint32_t c)
{
    // a 12-byte store (clang widens vec3 stores to 16 bytes, so no C++ form is safe here)
    const u32x3 v{a, b, c};
    // s_nop: the hazard recognizer does not see inside inline asm (a VALU write of the store's
    // data registers right after a >64-bit store needs a wait state)
    asm volatile("global_store_dwordx3 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void store_dwords(uint8_t *dst, u32x4 v, uint32_t lo, uint32_t hi)
{
    const u32x4 w = rot_down(v, lo >> 2);
    const uint32_t n = (hi - lo) >> 2;
    uint8_t *p = dst + lo;
    if (n == 3u) st12(p, w.x, w.y, w.z);
    else if (n == 2u) st8(p, w.x, w.y);
    else if (n == 1u) st4(p, w.x);
    else st16u_nt(p, w);
}

__device__ __noinline__ void store_bytes(uint8_t *dst, u32x4 v, uint32_t lo, uint32_t hi)
{
    // bytes [lo, hi) of the 16-byte register chunk v to dst + (lo..hi); rare path
    for (uint32_t b = lo; b < hi; b++) st1(dst + b, (uint8_t)(v[b >> 2] >> (8u * (b & 3u))));
}

// Store the payload part of datagram chunk c (bytes [16c, 16c+16) of the slot) to its
// place in the event: whole 16-byte stores inside the payload, whole dwords at the two
// edges, bytes only for a sub-dword event tail or a non dword-congruent datagram.
__device__ __forceinline__ void scatter_chunk(const PktInfo pi, uint32_t c, u32x4 v)
{
    if (pi.plen == 0) return;
    // datagram bytes [16c, 16c+16) against the payload [hl, hl+plen)
    const uint32_t q0 = 16u * c;
    const uint32_t pend = pi.hl + pi.plen;
    if (q0 >= pend || q0 + 16u <= pi.hl) return;
    const uint32_t lo = (q0 < pi.hl) ? pi.hl - q0 : 0u;             // first chunk byte to keep
    const uint32_t hi = (q0 + 16u <= pend) ? 16u : pend - q0;        // one past the last
    uint8_t *dst = reinterpret_cast<uint8_t *>(pi.dst) + q0 - pi.hl;  // where chunk byte 0 goes
    const bool congruent = ((pi.dst - pi.hl) & 3u) == 0;
    if (lo == 0 && hi == 16u && congruent) {
        st16u_nt(dst, v);
    } else if (congruent) {
        const uint32_t l4 = (lo + 3u) & ~3u, t = hi & ~3u;         // lo is a multiple of 4 here
        if (l4 < t) store_dwords(dst, v, l4, t);
        if (t < hi && t >= lo) store_bytes(dst, v, t, hi);         // sub-dword event tail
    } else {
        store_bytes(dst, v, lo, hi);
    }
}

__device__ __forceinline__ PktInfo ld_info(const PktInfo *p)
{
    const u32x4 v = *(const E2SAR_GLOBAL u32x4 *)(p);
    PktInfo r;
    r.dst = ((uint64_t)v.y << 32) | v.x;
    r.plen = v.z;
    r.hl = v.w;
    return r;
}

// Destination-aligned form of the same copy: chunk c of a payload whose phase in its event
// buffer is a (= bufferOffset mod 16; event buffers are 256-byte aligned in a 256-byte
// aligned arena) covers event bytes [(dst & ~15) + 16c, +16), i.e. datagram bytes from
// r = hl + 16c - a -- a multiple of 4 for a dword-congruent payload, so one dword-aligned
// 16-byte load, slid back by sh inside the slot at its end and shifted down in registers,
// feeds one aligned 16-byte store.
__device__ __forceinline__ uint32_t da_window(uint32_t c, uint32_t a, uint32_t hl, uint32_t stride, uint32_t &sh)
{
    const uint32_t r = hl + 16u * c - a;
    sh = (r + 16u > stride) ? r + 16u - stride : 0u;
    return r - sh;
}

// Store destination-aligned chunk c (loaded from the window of da_window) of the datagram
// at dgram: whole aligned 16-byte stores inside the payload, dwords at its two edges,
// bytes for a sub-dword event tail, byte copies for a payload that is not dword-congruent.
template <bool HO = false>
__device__ __forceinline__ void da_store(const PktInfo pi, uint32_t c, u32x4 x, const uint8_t *dgram, uint32_t stride)
{
    const uint32_t a = (uint32_t)pi.dst & 15u;
    if (pi.plen == 0u || 16u * c >= a + pi.plen) return;          // dropped, or past the payload
    uint8_t *D = reinterpret_cast<uint8_t *>((pi.dst & ~15ull) + 16ull * c);
    const uint32_t lo = (c == 0u) ? a : 0u;
    const uint32_t hi = (a + pi.plen - 16u * c < 16u) ? a + pi.plen - 16u * c : 16u;
    if ((a & 3u) == 0u) {
        uint32_t sh;
        (void)da_window(c, a, pi.hl, stride, sh);
        const u32x4 o = rot_down(x, sh >> 2);
        if (lo == 0u && hi == 16u) {
            st16_nt(D, o);
        } else {
            const uint32_t t = hi & ~3u;                               // lo = a is a multiple of 4
            if (lo < t) store_dwords(D, o, lo, t);
            if (t < hi && t >= lo) store_bytes(D, o, t, hi);           // sub-dword event tail
        }
    } else {
        const uint8_t *s = dgram + pi.hl + 16u * c - a;                // + lo >= hl
        for (uint32_t b = lo; b < hi; b++) st1(D + b, HO ? ld1_sc1(s + b) : ld1(s + b));
    }
}

// The fused kernel's store windows start on this many 16-byte blocks (one 128-byte line)
constexpr uint32_t kWinAlign = 8;

// Per-workgroup LDS of the fused reassembly: destinations of the group's datagrams, and
// the run tails' completion state (only the atomic's return value stays in registers during
// the copy, which keeps the kernel's occupancy up).
struct ReasGroupLds {
    PktInfo info[64];
    uint64_t ev[64], boff[64];
    uint32_t slot[64], bytes[64], d[64], rb[64], rc[64], tail[64];
};

// One group of gn <= 64 consecutive datagrams [g*G, g*G + gn), by the whole workgroup:
//   1. every wave loads the group's headers (lane p: datagram p); the load geometry of each
//      payload -- its phase in the event buffer and its length -- comes from them;
//   2. every thread issues its first U destination-aligned 16-byte payload loads;
//   3. wave 0 classifies (event table lookup/insert, run sums, counter atomics) while those
//      loads are in flight, and leaves each datagram's destination in LDS;
//   4. every thread stores its chunks (da_store), then loads and stores the rest round by
//      round (U chunks of 16 bytes per thread per round);
//   5. the run tails complete events (their atomic results are consumed last).
// HO: the chained form -- every datagram byte and length is read with sc1 loads (they were
// stored write-through by seg_block in the same launch).
template <int U, bool HO = false, int NT = kBlock>
__device__ __forceinline__ void reas_range(const ReasDev &R, const uint8_t *__restrict__ pkts, uint32_t stride,
                                           const uint32_t *__restrict__ lens, uint32_t g0, uint32_t gn, uint64_t now,
                                           uint32_t g, ReasGroupLds &L)
{
    const uint32_t tx = threadIdx.x;
    const bool w0 = tx < 64;
    const uint32_t lane = tx & 63u;

    TRACE_AT(0, 0, trace_now());
    // every wave issues the (cached) header loads so no load result crosses a branch
    const RawHdr raw = load_hdr<HO>(R, pkts, stride, lens, g0 + ((lane < gn) ? lane : 0u));
    TRACE_WAIT();
    TRACE_AT(2, 0, trace_now());

    // Index space: datagram p owns S = spc + 14 rounded down to 8 positions, and its
    // destination-aligned chunk c sits at position p * S + f + c, f = its destination's
    // 16-byte block within a 128-byte line (dst mod 128 = bufferOffset mod 128: event
    // buffers are 256-byte aligned).  Position ≡ destination block (mod 8), so every wave's
    // 64 positions store whole 128-byte lines at both ends of its window.  With one position
    // per chunk (S = spc), a window started and ended inside a line, the neighbouring
    // window's store instruction wrote the rest later, and the non-temporal lines left L2 in
    // between: 1.044x the payload in writes, 103 K partial write requests per launch; here
    // 1.003x and 16 K (profiles/round6/window_align/: reas_kernel at MTU 9000 68.2-68.8 vs
    // 69.9-70.8 us, at 1500 72.0-73.4 vs 72.8-74.6).  At MTU 1500 the padding costs no
    // round: 59 datagrams fill 1.77 rounds of 3072 chunks at S = 92 and 2.0 at S = 104.
    const uint32_t spc = stride >> 4;
    const uint32_t S = (spc + 2u * (kWinAlign - 1u)) & ~(kWinAlign - 1u);
    const uint32_t nch = gn * S;
    const float rS = 1.0f / (float)S;
    const uint8_t *const bpk = pkts + (uint64_t)g0 * stride;
    const __amdgpu_buffer_rsrc_t bpkR = brsrc(bpk);                     // HO loads only
    (void)bpkR;
    // position i -> (datagram, position within its S); recomputed at store time rather than
    // kept live across the classification (register pressure sets this kernel's occupancy)
    auto split_pos = [&](uint32_t i, uint32_t &p, uint32_t &j) {
        const uint32_t ic = (i < nch) ? i : 0u;
        p = (uint32_t)((float)ic * rS);
        if (p * S > ic) p--;
        else if ((p + 1u) * S <= ic) p++;
        j = ic - p * S;
    };
    const uint32_t hl = R.withLB ? kLBREHdrLen : kREHdrLen;
    const uint32_t gPhase = bswap32(raw.re.y) & (16u * kWinAlign - 1u);   // dst mod 128
    uint32_t gPlen = (raw.len >= hl) ? ((raw.len < stride) ? raw.len : stride) - hl : 0u;
    if (R.ownWorld > 1u && re_valid(raw.re.x) &&
        foreign_event(R, ((uint64_t)bswap32(raw.re.w) << 32) | bswap32(raw.re4)))
        gPlen = 0u;                                                    // another rank's: no payload loads
    auto issue = [&](uint32_t r0, u32x4(&xs)[U]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = r0 + (uint32_t)u * NT + tx;
            uint32_t p, j;
            split_pos(i, p, j);
            const uint32_t ph = __shfl(gPhase, (int)p), plen = __shfl(gPlen, (int)p);
            const uint32_t a = ph & 15u, f = ph >> 4, c = j - f;
            uint32_t off = 0, sh;
            if (i < nch && j >= f && 16u * c < a + plen && (a & 3u) == 0u) off = p * stride + da_window(c, a, hl, stride, sh);
            xs[u] = HO ? ld16_sc1(bpkR, off) : ld16(bpk + off);
        }
    };
    auto store = [&](uint32_t r0, const u32x4(&xs)[U]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = r0 + (uint32_t)u * NT + tx;
            if (i >= nch) continue;
            uint32_t p, j;
            split_pos(i, p, j);
            const PktInfo pi = L.info[p];
            const uint32_t f = ((uint32_t)pi.dst >> 4) & (kWinAlign - 1u);
            if (j < f) continue;
            da_store<HO>(pi, j - f, xs[u], bpk + (uint64_t)p * stride, stride);
        }
    };
    u32x4 x[U], y[U];
    // round 0 is in flight while wave 0 classifies.  (A/B, round 4: the first residency
    // wave's groups classifying before their round-0 loads, so their claims do not queue
    // behind 25 MB of loads, ran 0.5-2 us slower; round 1's loads in flight too -- the
    // pipeline's second register set live across the classification -- cut occupancy and
    // lost: DESIGN 4.5.)
    issue(0u, x);

    unsigned long long old = 0;
    if (w0) {
        const Classified cl = classify_wave<true>(R, raw, stride, lane < gn, now, g);
        L.info[lane] = cl.info;
        old = cl.old;
        L.ev[lane] = cl.ev;
        L.boff[lane] = cl.boff;
        L.slot[lane] = cl.slot;
        L.bytes[lane] = cl.sbytes;
        L.d[lane] = cl.d;
        L.rb[lane] = cl.rb;
        L.rc[lane] = cl.rc;
        L.tail[lane] = cl.tailAdd ? 1u : 0u;
        TRACE_AT(0, 1, trace_now());
    }
    lds_barrier();
    TRACE_AT(0, 2, trace_hwid());

    // software pipeline: the loads of round r+1 are issued before the stores of round r.
    // Loads, stores and atomics retire from vmcnt in issue order, so a load issued after
    // a store can only be waited for together with that store's write acknowledgement;
    // issued before it, round r+1's data is waited for while round r's stores drain.
    constexpr uint32_t RS = (uint32_t)(NT * U);
    if (RS < nch) issue(RS, y);
    store(0u, x);
    for (uint32_t r0 = RS; r0 < nch; r0 += 2 * RS) {
        if (r0 + RS < nch) issue(r0 + RS, x);
        store(r0, y);
        if (r0 + RS >= nch) break;
        if (r0 + 2 * RS < nch) issue(r0 + 2 * RS, y);
        store(r0 + RS, x);
    }

    if (w0 && L.tail[lane]) {
        Classified cl;
        // in-order vmcnt: issued before the copy, this atomic's return (slow when ~100 groups
        // of one event add at once) would gate wave 0's first copy wait
        if (L.bytes[lane] >= kDeferAccBytes)
            old = atomicAdd(&R.slots[L.slot[lane]].acc, ((unsigned long long)L.rc[lane] << kAccFragShift) | L.rb[lane]);
        cl.old = old;
        cl.ev = L.ev[lane];
        cl.boff = L.boff[lane];
        cl.slot = L.slot[lane];
        cl.sbytes = L.bytes[lane];
        cl.d = L.d[lane];
        cl.rb = L.rb[lane];
        cl.rc = L.rc[lane];
        cl.tailAdd = true;
        classify_finish(R, cl);
    }
#if E2SAR_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    TRACE_AT(0, 3, trace_now());
#endif
}

// starts (optional): group g is datagrams [starts[g], starts[g+1]) (<= 64), e.g. the XCD
// stripes of the batch's segmentation (seg_groups); otherwise [g*G, g*G + G).
template <int U, bool HO = false, int NT = kBlock>
__device__ __forceinline__ void reas_group(const ReasDev &R, const uint8_t *__restrict__ pkts, uint32_t stride,
                                           const uint32_t *__restrict__ lens, uint32_t n, uint64_t now, uint32_t G,
                                           uint32_t g, ReasGroupLds &L, const uint32_t *__restrict__ starts = nullptr)
{
    uint32_t g0 = g * G;
    uint32_t gn = (n - g0 < G) ? n - g0 : G;
    if (starts) {
        // a caller-supplied device table: never trust it past the batch
        g0 = starts[g];
        if (g0 >= n) return;
        const uint32_t g1 = (starts[g + 1] < n) ? starts[g + 1] : n;
        if (g1 <= g0 || g1 - g0 > 64u) return;                       // empty or oversized group
        gn = g1 - g0;
    }
    reas_range<U, HO, NT>(R, pkts, stride, lens, g0, gn, now, g, L);
}

// reas_kernel: workgroup b reassembles datagrams [b*G, b*G + G) of the batch.
// (A/B: a resident grid drawing groups dynamically from per-XCD work counters, to even
// out XCDs that stream at different rates, ran 1.7-2.2x slower: a workgroup's groups are
// then classified one after another and every classification -- ~7 us of dependent table
// round trips -- sits in front of its copy, where the one-shot grid classifies all groups
// at once while the first round of loads is in flight.  Round 2 gave the resident grid a
// classifier wave that classifies the next group while copy waves copy the current one,
// then an LDS ring of classified groups: bit-exact, 79.7-81.8 us against 74-75 us here --
// the groups buffered per workgroup when the queues run dry lengthen the tail)
// NT threads per workgroup: wave 0 classifies while all NT/64 waves hold a round of loads
// (NT x U chunks) in flight.  Round 4 (profiles/round4/ab/reas_threads.log,
// reas_group_sizes.log): 768 threads (two workgroups of 12 waves per CU, 59-datagram
// groups in 1.8 rounds) take the 1 MiB @ MTU 1500 batch in 72.7-72.9 us against 75.4-75.7
// at 256 (six of 4 waves, 49 datagrams in 4.4 rounds); with jumbo slots 512 threads do
// best (71.0 against 73.4-74.0 us at 256 and 71.7 at 768); 1024 threads (one workgroup
// per CU) lose (82-84 us).
template <int U, int NT>
__global__ __launch_bounds__(NT) void reas_kernel(ReasDev R, const uint8_t *__restrict__ pkts, uint32_t stride,
                                                  const uint32_t *__restrict__ lens, uint32_t n, uint64_t now,
                                                  uint32_t G, const uint32_t *__restrict__ starts)
{
    __shared__ ReasGroupLds L;
    reas_group<U, false, NT>(R, pkts, stride, lens, n, now, G, blockIdx.x, L, starts);
}

// reas_kernel's workgroup size for a slot stride
constexpr int kReasNTSmall = 768;   // slots of <= 4 KiB
constexpr int kReasNTJumbo = 512;
__host__ __device__ constexpr int reas_threads(uint32_t stride)
{
    return stride <= 4096u ? kReasNTSmall : kReasNTJumbo;
}

// ---------------------------------------------------------------------------------
// chained form: segmentation of a batch and reassembly of the same datagrams in ONE launch.
// Workgroups [0, nSeg) are seg_kernel blocks (HO: write-through stores, then a per-group
// counter add); workgroups [nSeg, nSeg + groups) are reas_kernel groups, each of which
// waits until its counter shows every datagram of its range written, then runs as in
// reas_kernel with sc1 loads.  A group waits only on blocks with lower indices, which
// are dispatched before it and never wait, so the grid always drains; the wait is also
// bounded (2 s, error flag bit 4), so a miscount can never hang the device.  The group
// resets its counter for the next launch.  What this buys over two launches: the
// reassembly groups start while the last segmentation blocks finish (no kernel boundary,
// no half-empty tail between the two kernels).

#if E2SAR_HIP_EXPERIMENTAL
// seg blocks of 16 KiB (8-KiB blocks, as seg_kernel uses for 1 MiB events, made the chained
// launch 147 -> 158 us: twice the blocks at the reassembly occupancy)
constexpr int kChainSegU = 4;

__device__ __forceinline__ void wait_group_ready(const ReasDev &R, uint32_t *tiles, uint32_t g, uint32_t expect)
{
    if (threadIdx.x == 0) {
        uint32_t *t = tiles + g;
        uint64_t t0 = 0;
        for (uint32_t it = 0;; it++) {
            const uint32_t v = ld4_sc1(t);
            if (v >= expect) {
                if (v != expect) atomicOr(&R.ctl->errorFlags, 32u);           // over-count
                break;
            }
            const uint64_t now = __builtin_amdgcn_s_memrealtime();           // 100 MHz
            if (it == 0) t0 = now;
            else if (now - t0 > 200000000ull) {
                atomicOr(&R.ctl->errorFlags, 16u);                           // wait timed out
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        st4_sc1(t, 0u);
    }
    __syncthreads();
}

template <int U>
__global__ __launch_bounds__(kBlock) void segreas_kernel(ChainBatches cb, int lbVersion,
                                                                              uint32_t maxPld, uint32_t stride,
                                                                              ReasDev R, uint64_t now)
{
    __shared__ ReasGroupLds L;
    // grid: [seg(0) | reas(0) | seg(1) | reas(1) | ...]; a reassembly group depends only on
    // segmentation blocks of its own batch, all of which have lower indices
    uint32_t b = 0;
    while (b + 1u < cb.nb && blockIdx.x >= cb.b[b + 1u].start) b++;
    const ChainBatch &B = cb.b[b];
    const uint32_t local = blockIdx.x - B.start;
    if (local < B.nSeg) {
        seg_block<kChainSegU, true>(B.events, B.bpe, lbVersion, maxPld, B.pkts, stride, B.lens, nullptr, local,
                                           B.G, B.tiles);
        return;
    }
    const uint32_t g = local - B.nSeg;
    const uint32_t slots = (B.n - g * B.G < B.G) ? B.n - g * B.G : B.G;
    wait_group_ready(R, B.tiles, g, slots * (stride >> 4));
    reas_group<U, true>(R, B.pkts, stride, B.lens, B.n, now, B.G, g, L);
}

#endif  // E2SAR_HIP_EXPERIMENTAL

// ---------------------------------------------------------------------------------
// reassembly as two phases: classify (headers only, latency-bound) then scatter (bytes
// only, bandwidth-bound).  Each phase is a launch of its own, or -- the pipelined form --
// one launch scatters batch b while other workgroups of the same grid classify batch
// b+1, so the table round trips of b+1 run under the copy of b instead of in front of it.
//
// Work buffer of a classified batch of n datagrams: PktInfo[n] then FinishRec[n].  A run
// tail whose add completed its event sets kPktCompletes in its own PktInfo.hl and writes
// FinishRec[p]; the scatter workgroup that owns datagram p publishes the event after its
// own stores (the bytes of every workgroup are visible at the end of that launch).

constexpr uint32_t kPktCompletes = 0x80000000u;
constexpr uint32_t kFinKeepSlot = 0x80000000u;     // FinishRec.slot flag (reference-order mode)

// One wave: classify datagrams [p0, p0+64) of the batch.
__device__ __forceinline__ void classify_wave_to_work(const ReasDev &R, const uint8_t *__restrict__ pkts,
                                                      uint32_t stride, const uint32_t *__restrict__ lens,
                                                      uint32_t n, uint64_t now, PktInfo *__restrict__ info,
                                                      FinishRec *__restrict__ fin, uint32_t wave)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t p0 = wave * 64u;
    if (p0 >= n) return;                                       // wave-uniform
    const uint32_t gn = (n - p0 < 64u) ? n - p0 : 64u;
    const RawHdr raw = load_hdr(R, pkts, stride, lens, p0 + ((lane < gn) ? lane : 0u));
    const Classified cl = classify_wave(R, raw, stride, lane < gn, now, wave);
    const bool done = completes(cl);
    if (lane < gn) {
        const u32x4 v = {(uint32_t)cl.info.dst, (uint32_t)(cl.info.dst >> 32), cl.info.plen,
                         cl.info.hl | (done ? kPktCompletes : 0u)};
        st16(reinterpret_cast<uint8_t *>(info + p0 + lane), v);
    }
    if (done) {
        FinishRec f;
        f.ev = cl.ev;
        f.boff = cl.boff;
        f.slot = cl.slot;
        f.bytes = cl.sbytes;
        f.frags = (uint32_t)(cl.old >> kAccFragShift) + cl.rc;
        f.d = cl.d;
        fin[p0 + lane] = f;
    }
}

// Scatter stores: source-aligned chunks, staged through LDS into aligned stores
// (lds_stage_store) where scatter_stage() picks it, else stored at their misaligned
// destination (scatter_chunk).  (Round 3 measured destination-aligned stores built from
// neighbour-lane funnel shifts, or from every lane loading its chunk pair: cold leg 2221 /
// 2020 vs 2369 GiB/s -- what the aligned stores save the extra loads cost)

// Staged scatter (STAGE, chosen per launch by scatter_stage()): the one-round group's
// source-aligned chunks go through LDS.  Every dword of a payload is written to its destination phase in the group's LDS
// copy of the slot (datagram p at p * (stride + 16), payload byte t at a + t, a = dst mod
// 16), then after an LDS barrier every 16-byte event block is read back aligned and stored
// aligned: the loads need nothing from the work records, the stores are whole aligned
// 16-byte stores except at the payload's two edges.  A payload that is not dword-congruent
// with its destination (never at dword-multiple maxPld) is stored from registers as before.
template <int U, int TB>
__device__ __forceinline__ void lds_stage_store(const PktInfo *sinfo, const u32x4 (&x)[U], const uint32_t (&pp)[U],
                                                const uint32_t (&cc)[U], uint32_t nch, uint32_t gn, uint32_t stride)
{
    // one round of the group's slots (<= 256 * U chunks) plus 16 bytes of phase per datagram
    __shared__ uint32_t stage[(16u * TB * U + 64u * 16u) / 4u];
    const uint32_t ps = stride + 16u;                                  // LDS bytes per datagram
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t i = (uint32_t)u * TB + threadIdx.x;
        if (i >= nch) continue;
        const PktInfo pi = sinfo[pp[u]];
        if (pi.plen == 0u) continue;
        const uint32_t a = (uint32_t)pi.dst & 15u;
        if (((a - pi.hl) & 3u) != 0u) {                                // not dword-congruent
            scatter_chunk(pi, cc[u], x[u]);
            continue;
        }
        const uint32_t base = pp[u] * ps + a - pi.hl;                  // + slot byte offset
#pragma unroll
        for (uint32_t d = 0; d < 4; d++) {
            const uint32_t s = 16u * cc[u] + 4u * d;
            if (s >= pi.hl && s < pi.hl + pi.plen) stage[(base + s) >> 2] = x[u][d];
        }
    }
    lds_barrier();
    const uint32_t nbp = ps >> 4;                                      // 16-byte blocks per datagram
    const uint32_t total = gn * nbp;
    for (uint32_t k = threadIdx.x; k < total; k += TB) {
        const uint32_t p = k / nbp, b = k - p * nbp;
        const PktInfo pi = sinfo[p];
        if (pi.plen == 0u) continue;
        const uint32_t a = (uint32_t)pi.dst & 15u;
        if (((a - pi.hl) & 3u) != 0u || 16u * b >= a + pi.plen) continue;
        const uint32_t q = (p * ps + 16u * b) >> 2;
        const u32x4 o{stage[q], stage[q + 1], stage[q + 2], stage[q + 3]};
        uint8_t *D = reinterpret_cast<uint8_t *>((pi.dst & ~15ull) + 16ull * b);
        const uint32_t lo = (b == 0u) ? a : 0u;
        const uint32_t hi = (a + pi.plen - 16u * b < 16u) ? a + pi.plen - 16u * b : 16u;
        if (lo == 0u && hi == 16u) {
            st16_nt(D, o);
            continue;
        }
#pragma unroll
        for (uint32_t d = 0; d < 4; d++)
            if (4u * d >= lo && 4u * d + 4u <= hi) st4(D + 4u * d, o[d]);
        const uint32_t t = hi & ~3u;                                   // sub-dword event tail
        if (t < hi && t >= lo) store_bytes(D, o, t, hi);
    }
}

// One workgroup: scatter datagrams [blk*G, blk*G+G) of a classified batch.
template <int U, bool NT, bool STAGE, int TB>
__device__ __forceinline__ void scatter_group(const ReasDev &R, const uint8_t *__restrict__ pkts, uint32_t stride,
                                              uint32_t n, uint32_t G, const PktInfo *__restrict__ info,
                                              const FinishRec *__restrict__ fin, uint32_t blk, PktInfo *sinfo)
{
    const uint32_t g0 = blk * G;
    const uint32_t gn = (n - g0 < G) ? n - g0 : G;
    const uint32_t lane = threadIdx.x & 63u;

    // every wave loads the records (cached) so no load result crosses a branch; they are
    // issued before the payload loads so waiting for them does not wait for the payload
    const PktInfo mine = ld_info(info + g0 + ((lane < gn) ? lane : 0u));

    const uint32_t spc = stride >> 4;
    uint32_t nch = gn * spc;
    const float rspc = 1.0f / (float)spc;
    const uint8_t *const bpk = pkts + (uint64_t)g0 * stride;
    u32x4 x[U];
    uint32_t pp[U], cc[U];
    auto issue = [&](uint32_t r0) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = r0 + (uint32_t)u * TB + threadIdx.x;
            const uint32_t ic = (i < nch) ? i : 0u;
            uint32_t p = (uint32_t)((float)ic * rspc);
            if (p * spc > ic) p--;
            else if ((p + 1u) * spc <= ic) p++;
            pp[u] = p;
            cc[u] = ic - p * spc;
            const uint8_t *src = bpk + (uint64_t)p * stride + 16u * cc[u];
            x[u] = NT ? ld16_nt(src) : ld16(src);
        }
    };
    issue(0);
    bool fins = false;
    if (threadIdx.x < 64) {
        // a record that does not land inside the arena (a work buffer that was not filled
        // by classify for this batch) is dropped and flagged, never written through
        const uint64_t lo = (uint64_t)R.arena, hi = lo + R.arenaBytes;
        const bool inside = mine.plen == 0 || (mine.dst >= lo && mine.dst + mine.plen <= hi);
        if (lane < gn && !inside) atomicOr(&R.ctl->errorFlags, 8u);
        PktInfo v = (lane < gn && inside) ? mine : PktInfo{0ull, 0u, 0u};
        fins = (v.hl & kPktCompletes) != 0u;
        v.hl &= ~kPktCompletes;
        sinfo[lane] = v;
    }
    __syncthreads();

    if constexpr (STAGE) {
        if (nch <= (uint32_t)(TB * U)) {
            lds_stage_store<U, TB>(sinfo, x, pp, cc, nch, gn, stride);
            nch = 0;                                                 // done: skip the rounds below
        }
    }
    for (uint32_t r0 = 0; r0 < nch; r0 += (uint32_t)(TB * U)) {
        if (r0) issue(r0);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = r0 + (uint32_t)u * TB + threadIdx.x;
            if (i >= nch) continue;
            scatter_chunk(sinfo[pp[u]], cc[u], x[u]);
        }
    }

    if (fins) {
        const FinishRec f = fin[g0 + lane];
        const uint32_t fs = f.slot & ~kFinKeepSlot;
        if (fs < R.tableSlots) complete_event(R, fs, f.ev, f.boff, f.bytes, f.d, f.frags, (f.slot & kFinKeepSlot) != 0u);
        else atomicOr(&R.ctl->errorFlags, 8u);
    }
}

// (Round 3-4: chunk-range scatter workgroups -- loads exactly a linear 16-KiB range of the
// slots whatever datagrams they belong to, registers or LDS-staged -- measured no better on
// config 3 and lost on the cold leg; removed)

// XCD-aware visit order of the scatter forms (round 5).  Workgroup b of a launch runs on XCD
// b mod 8 (round-robin dispatch; a speed assumption only, never correctness).  In dispatch
// order, consecutive scatter groups -- one 8976-byte datagram at MTU 9000, eight at 1500 --
// sat on different XCDs, so every group boundary (a 128-byte slot line shared by two
// datagrams, and at the destination a line shared by two payloads) was touched by two
// XCDs' L2s.  Here each XCD takes runs of kXcdRun consecutive groups, the eight XCDs' runs
// side by side, so the launch still moves through the batch as one front.  Config 3 (70 x 8
// MiB at MTU 9000, 65,730 one-datagram groups): split reassembly 231-234 -> 211-213 us with
// runs of 128 (32-128 within 2 us; 8 or 16 contiguous regions, one per XCD, 221-224 us;
// spreading the groups in flight over 64-70 regions 236-246 us), cold leg at MTU 1500
// unchanged within noise (profiles/round5/xcd_order/).  A bijection on [0, nb): the last
// nb mod (8 kXcdRun) groups keep their order.
constexpr uint32_t kXcdRun = 128;
__host__ __device__ constexpr uint32_t xcd_runs(uint32_t b, uint32_t nb)
{
    constexpr uint32_t W = 8u * kXcdRun;
    if (b >= nb / W * W) return b;
    const uint32_t w = b % W;
    return (b - w) + (w % 8u) * kXcdRun + w / 8u;
}
// every group is visited exactly once (checked at compile time around the window edges)
constexpr bool xcd_runs_bijective(uint32_t nb)
{
    bool seen[3200] = {};
    for (uint32_t b = 0; b < nb; b++) {
        const uint32_t g = xcd_runs(b, nb);
        if (g >= nb || seen[g]) return false;
        seen[g] = true;
    }
    return true;
}
static_assert(xcd_runs_bijective(1) && xcd_runs_bijective(1023) && xcd_runs_bijective(1024) &&
                  xcd_runs_bijective(1025) && xcd_runs_bijective(2048) && xcd_runs_bijective(3199),
              "xcd_runs must be a bijection on [0, nb)");

__global__ __launch_bounds__(kBlock) void reas_classify_kernel(ReasDev R, const uint8_t *__restrict__ pkts,
                                                               uint32_t stride, const uint32_t *__restrict__ lens,
                                                               uint32_t n, uint64_t now, PktInfo *__restrict__ info,
                                                               FinishRec *__restrict__ fin)
{
    classify_wave_to_work(R, pkts, stride, lens, n, now, info, fin, blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6));
}

template <int U, bool NT, bool STAGE, int TB = kScatBlock>
__global__ __launch_bounds__(TB) void reas_scatter_kernel(ReasDev R, const uint8_t *__restrict__ pkts,
                                                              uint32_t stride, uint32_t n, uint32_t G,
                                                              const PktInfo *__restrict__ info,
                                                              const FinishRec *__restrict__ fin)
{
    __shared__ PktInfo sinfo[64];
    scatter_group<U, NT, STAGE, TB>(R, pkts, stride, n, G, info, fin, xcd_runs(blockIdx.x, (n + G - 1u) / G), sinfo);
}

// Pipelined form: workgroups [clsStart, clsStart + nClsBlocks) classify batch b+1, the rest
// scatter batch b (in xcd_runs order: clsStart and nClsBlocks are multiples of 8, so a
// scatter workgroup's index keeps its XCD parity).
template <int U, bool NT, bool STAGE, int TB = kScatBlock>
__global__ __launch_bounds__(TB) void reas_scatter_classify_kernel(
    ReasDev R, uint32_t stride, const uint8_t *__restrict__ spk, uint32_t sn, uint32_t G,
    const PktInfo *__restrict__ sinfoG, const FinishRec *__restrict__ sfin, const uint8_t *__restrict__ cpk,
    const uint32_t *__restrict__ clens, uint32_t cn, uint64_t now, PktInfo *__restrict__ cinfo,
    FinishRec *__restrict__ cfin, uint32_t nClsBlocks, uint32_t clsStart)
{
    __shared__ PktInfo sinfo[64];
    // workgroups [clsStart, clsStart + nClsBlocks) classify, the others scatter
    const uint32_t b = blockIdx.x;
    if (b - clsStart < nClsBlocks) {
        classify_wave_to_work(R, cpk, stride, clens, cn, now, cinfo, cfin,
                              (b - clsStart) * (TB / 64) + (threadIdx.x >> 6));
        return;
    }
    const uint32_t sb = (b < clsStart) ? b : b - nClsBlocks;
    scatter_group<U, NT, STAGE, TB>(R, spk, stride, sn, G, sinfoG, sfin, xcd_runs(sb, (sn + G - 1u) / G), sinfo);
}

// ---------------------------------------------------------------------------------
// reassembly in the reference's arrival order (E2SAR_HIP_REAS_REFERENCE_ORDER)
//
// The reference's receive body takes datagrams one at a time (e2sarDPReassembler.cpp:
// 335-427), and for some inputs the order decides the outcome: a fragment with
// bufferOffset 0 always starts a new item, replacing (dropping) an item in progress under
// the same key (cpp:361-369); a fragment whose key has no item starts one (cpp:376-384),
// also after its event completed; completion is tested after every fragment (cpp:403), so
// a duplicate that arrives before the last fragment makes curBytes overshoot while one that
// arrives after completion starts an item of its own.  This mode reproduces that for any
// arrival order (batch order, then datagram order within a batch):
//   ro_key_kernel  : parse and validate every datagram (counters as classify_wave), register
//                    its key in the table (find_or_create<keyOnly>), write a 16-byte record
//                    {off, plen, blen, hl}, and file every run of consecutive positions of
//                    one key (per wave) in the key's bucket of kRoBucket runs (past that in
//                    an overflow list); a key's first run lists the key;
//   ro_place_kernel: one workgroup: hands the number of listed keys to the walk and resets
//                    the counters; only if a key overflowed its bucket, places and sorts by
//                    position the runs of every such key;
//   ro_walk_kernel : one wave per key orders its runs by position (rank and push, <= 64 runs) and
//                    walks that key's datagrams in arrival order with the reference's rules,
//                    creating items (arena buffers) as it goes, and writes the PktInfo /
//                    FinishRec work records of the split form;
//   reas_scatter_kernel then moves the bytes and publishes the completions.

// key of a datagram that does not take part (bad header, bounds, table full): no real slot,
// so it joins no run
constexpr uint32_t kRoNoSlot = 0xFFFFFFFFu;
// Key-pass workgroup: 1024 threads (round 6, profiles/round6/ro_keypass/): events
// interleaved datagram by datagram put the same keys in every workgroup of their span, and
// each workgroup registers a key and files its runs with one lookup and one returning atomic
// on that key's slot -- 1024-datagram workgroups make 4x fewer of those than 256: K = 64 /
// 205 interleaved events 190 / 425 -> 135-137 / 232-235 us per batch, K = 1 / 8 91.7-94.0 /
// 117-118 -> 91.2-91.8 / 113-114 (512 threads: 144-146 / 290-292; 1024 threads with two
// datagrams per lane, one workgroup per CU: 148-149 / 237 -- too few workgroups).
constexpr int kRoKeyBlock = 1024;

template <int TB>
__global__ __launch_bounds__(TB) void ro_key_kernel(ReasDev R, const uint8_t *__restrict__ pkts, uint32_t stride,
                                                    const uint32_t *__restrict__ lens, uint32_t n, uint64_t now,
                                                    RoScratch sc, PktInfo *__restrict__ info)
{
    // the workgroup's distinct keys (at most TB): one global lookup and one run-count
    // atomic per key per workgroup, not per wave
    constexpr uint32_t kWgKeys = 2u * TB;       // the per-workgroup key table
    __shared__ unsigned long long wgEv[kWgKeys];
    __shared__ uint32_t wgD[kWgKeys], wgTag[kWgKeys], wgCnt[kWgKeys], wgSlot[kWgKeys], wgBase[kWgKeys];
    const uint32_t wave = blockIdx.x * (TB / 64) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t p0 = wave * 64u;
    const bool waveLive = p0 < n;                              // (a wave past n still meets the barriers)
    const uint32_t gn = !waveLive ? 0u : (n - p0 < 64u) ? n - p0 : 64u;
    const bool live = lane < gn;
    const uint32_t p = waveLive ? p0 + (live ? lane : 0u) : 0u;
    for (uint32_t i = threadIdx.x; i < kWgKeys; i += TB) {
        wgTag[i] = 0u;
        wgCnt[i] = 0u;
    }
    const RawHdr raw = load_hdr(R, pkts, stride, lens, p);
    const uint32_t hl = R.withLB ? kLBREHdrLen : kREHdrLen;
    ParsedHdr h = parse_hdr(raw, hl, stride, live);
    const bool foreign = h.ok && foreign_event(R, h.ev);      // another rank's event: takes no part
    if (foreign) h = ParsedHdr{0, 0, 0, 0, 0, false, false, false};
    // bounds against the fragment's own bufferLength, before the lookup (the reference
    // memcpy's unchecked at cpp:391; dropped and counted here)
    if (h.ok && (uint64_t)h.off + h.pl > h.blen) {
        h.ok = false;
        h.derr = true;
    }
    // runs of equal keys: only the run head takes part.  Every head registers its key in the
    // workgroup's table itself and takes its run index there with one LDS atomic (round 6:
    // a per-wave loop that first collapsed the heads of one key took 64 passes in a wave of
    // 64 interleaved events; K = 64 / 205 136.5 / 233 -> 126.5 / 225 us per batch, in
    // order unchanged, profiles/round6/ro_keypass/)
    const uint64_t pev = ((uint64_t)lane_prev((uint32_t)(h.ev >> 32), 0u) << 32) | lane_prev((uint32_t)h.ev, 0u);
    const uint32_t pd = lane_prev(h.d, 0u), pok = lane_prev(h.ok ? 1u : 0u, 0u);
    const bool head = h.ok && (lane == 0 || !pok || pev != h.ev || pd != h.d);
    // each head claims or finds its key's entry in the workgroup's table
    uint32_t e = slot_hash(h.ev, h.d, kWgKeys - 1u);
    bool pending = head, check = false;
    __syncthreads();                                           // table cleared
    while (__syncthreads_or(pending)) {
        if (pending) {
            if (atomicCAS(&wgTag[e], 0u, 1u) == 0u) {
                wgEv[e] = h.ev;
                wgD[e] = h.d;
                pending = false;
            } else {
                check = true;
            }
        }
        __syncthreads();                                       // claimed keys are written
        if (check) {
            check = false;
            if (wgEv[e] == h.ev && wgD[e] == h.d) pending = false;
            else e = (e + 1u) & (kWgKeys - 1u);
        }
    }
    // this head's run: its index among the workgroup's runs of the key
    uint32_t o = 0;
    if (head) o = atomicAdd(&wgCnt[e], 1u);
    __syncthreads();
    for (uint32_t b = 0; b < kWgKeys; b += TB) {               // one lookup + one atomic per key
        const uint32_t i = b + threadIdx.x;
        const bool want = wgTag[i] != 0u;
        const LookupResult lr = find_or_create<true>(R, want, wgEv[i], wgD[i], 0u, now);
        if (want) {
            wgSlot[i] = lr.slot;
            wgBase[i] = lr.slot != kNoSlot ? atomicAdd(&sc.runCnt[lr.slot], wgCnt[i]) : 0u;
        }
    }
    __syncthreads();
    const uint32_t hslot = head ? wgSlot[e] : kNoSlot;
    const uint32_t k = head ? wgBase[e] + o : 0u;            // this run's index in its key
    const uint64_t H = __ballot(head);
    const uint64_t le = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
    const uint64_t hm = H & le;
    const int myhead = hm ? 63 - __builtin_clzll(hm) : (int)lane;
    const uint32_t slot = __shfl(hslot, myhead);
    if (h.ok && slot == kNoSlot) {                             // table full / probe timeout
        h.ok = false;
        h.derr = true;
    }
    if (live) {
        const u32x4 v = {h.off, h.pl, h.blen, hl};
        st16(reinterpret_cast<uint8_t *>(sc.recs + p), v);
        if (!h.ok) st16(reinterpret_cast<uint8_t *>(info + p), u32x4{0u, 0u, 0u, hl});   // takes no part
    }
    // runs of consecutive positions of one key (one slot) within the wave -- they start at
    // the heads -- filed in the slot's bucket (the run of index 0 lists the slot for the walk)
    const uint32_t ks = h.ok ? slot : kRoNoSlot;
    const uint32_t pks = lane_prev(ks, kRoNoSlot), nks = lane_next(ks, kRoNoSlot);
    const bool rhead = h.ok && (lane == 0 || pks != ks);
    const bool rtail = h.ok && (lane == 63 || nks != ks);
    const uint64_t RT = __ballot(rtail);
    if (rhead) {
        const uint64_t below = (1ull << lane) - 1ull;
        const uint32_t len = (uint32_t)__builtin_ctzll(RT & ~below) - lane + 1u;   // to this run's last lane
        if (k == 0u) sc.active[atomicAdd(&sc.ctr[1], 1u)] = slot;
        if (k < kRoBucket) {
            sc.bucket[(size_t)slot * kRoBucket + k] = ((unsigned long long)p << 32) | len;
        } else {
            st16(reinterpret_cast<uint8_t *>(sc.runs + p), u32x4{slot, p, len, k});   // at its head's position
        }
    }
    // which lanes of this wave hold an overflow run (every wave writes its word; a flag tells
    // the place pass to look -- a plain store, not a counter all waves would contend on)
    const uint64_t OV = __ballot(rhead && k >= kRoBucket);
    if (lane == 0 && waveLive) {
        sc.ovMask[wave] = OV;
        if (OV) sc.ctr[0] = 1u;
    }
    wave_stats(R, live && !foreign, (live && !foreign) ? raw.len : 0u, h.bad, h.derr, wave);
}

// Between the key pass and the walk: hands the count of listed keys to the walk (ctr[1] ->
// ctr[2]) and resets it for the next batch (ctr[0] is reset by the walk: every workgroup
// here reads it).  Only when some key filed more than kRoBucket runs (ctr[0] set: events
// interleaved in arrival, or very large ones) does it do more: an exclusive scan of the run
// counts of those keys gives each its place (runBase), and every overflow run (found by the
// key-pass waves' overflow masks, stored at its head's position) is copied to runBase + its
// index in the key (k, from the key pass's count) -- no atomics, no order: the key's walk
// wave orders them.  Every workgroup computes the scan itself, into LDS (no grid
// synchronisation), and places a share of the runs; a table above kPlaceLdsSlots slots is
// handled by workgroup 0 alone through the global runBase.
constexpr uint32_t kPlaceThreads = 256, kPlaceBlocks = 64, kPlaceLdsSlots = 16384;
__global__ __launch_bounds__(kPlaceThreads) void ro_place_kernel(RoScratch sc, uint32_t T, uint32_t n)
{
    __shared__ uint32_t base[kPlaceLdsSlots];
    __shared__ uint32_t part[kPlaceThreads];
    const uint32_t t = threadIdx.x;
    const uint32_t nOver = sc.ctr[0];
    if (blockIdx.x == 0 && t == 0) {
        sc.ctr[2] = sc.ctr[1];
        sc.ctr[1] = 0u;
    }
    if (nOver == 0u) return;                                          // uniform: the usual case
    const bool inLds = T <= kPlaceLdsSlots;
    if (!inLds && blockIdx.x != 0) return;
    const uint32_t per = (T + kPlaceThreads - 1u) / kPlaceThreads;
    const uint32_t s0 = t * per < T ? t * per : T, s1 = s0 + per < T ? s0 + per : T;
    uint32_t sum = 0;
    for (uint32_t q = s0; q < s1; q++) {
        const uint32_t c = sc.runCnt[q];
        sum += c > kRoBucket ? c : 0u;
    }
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < kPlaceThreads; off <<= 1) {           // inclusive scan
        const uint32_t v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t b = part[t] - sum;
    for (uint32_t q = s0; q < s1; q++) {
        const uint32_t c = sc.runCnt[q];
        if (inLds) base[q] = b;
        if (blockIdx.x == 0) sc.runBase[q] = b;
        b += c > kRoBucket ? c : 0u;
    }
    __syncthreads();                        // (global runBase: written and read by this workgroup)
    // one thread per datagram position: an overflow run sits at its head's position, marked
    // in its key-pass wave's mask
    const uint32_t nThreads = inLds ? gridDim.x * kPlaceThreads : kPlaceThreads;
    for (uint32_t p = (inLds ? blockIdx.x * kPlaceThreads : 0u) + t; p < n; p += nThreads) {
        if ((sc.ovMask[p >> 6] >> (p & 63u)) & 1ull) {
            const u32x4 run = ld16(reinterpret_cast<const uint8_t *>(sc.runs + p));   // slot, start, len, k
            const uint32_t rb = inLds ? base[run.x] : sc.runBase[run.x];
            sc.placed[rb + run.w] = ((unsigned long long)run.y << 32) | run.z;
        }
    }
}

// One wave per key walks the key's datagrams in arrival order, 64 at a time, with the
// reference's rules (cpp:361-427).  The key's runs are taken 64 at a time in position order --
// a slot of at most kRoBucket runs orders its bucket here (rank by start, one lane push), a
// larger one was placed and sorted by ro_place_kernel -- and a datagram index of
// the concatenated runs maps to its position by a binary search over the runs' prefix sums.  The item state (buffer, length, curBytes, fragments) is
// wave-uniform.  Within a chunk the walk goes segment by segment: a segment starts where a
// new item starts (offset 0, or no item in progress) and runs to the next offset-0 fragment;
// a masked prefix sum of the payload lengths finds the first fragment whose add makes
// curBytes equal the item's length (completion, cpp:403), which ends the segment early.
// Fragments that overrun the item (made by a fragment with another bufferLength) count as
// data errors and add nothing.  One segment per chunk is the usual case; duplicates, late
// offset-0 fragments and replays after completion add segments.
constexpr uint32_t kRoAhead = 4;
constexpr uint32_t kRoSortLds = 2048;       // runs of one key sorted in LDS by its wave (16 KiB)
// The walk runs one wave per workgroup with 32 KiB of LDS (round 6, profiles/round6/ro_walk/):
// four key waves per workgroup sharing a CU, 16 KiB each, left three quarters of the CUs
// idle and sent keys whose span outgrew a 16 KiB position bitmap to the run sort -- 205
// events interleaved 224 -> 151 us per batch, in order and K = 8 / 64 about 1 us faster.
constexpr uint32_t kRoWalkLds = 4096;       // 8-byte words of LDS per walk wave

// Bitonic sort of P = 128 NP keys in LDS by one wave: per stage each lane loads its NP
// pairs at once (one LDS round trip per stage, not one per pair), then compares and stores.
template <int NP>
__device__ __forceinline__ void wave_sort_lds(unsigned long long *v, uint32_t lane)
{
    constexpr uint32_t P = 128u * NP;
    for (uint32_t k = 2; k <= P; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            unsigned long long x[NP], y[NP];
            uint32_t ii[NP];
#pragma unroll
            for (uint32_t t = 0; t < (uint32_t)NP; t++) {
                const uint32_t q = lane + 64u * t;                   // pair q: elements i, i + j
                ii[t] = ((q & ~(j - 1u)) << 1) | (q & (j - 1u));
                x[t] = v[ii[t]];
                y[t] = v[ii[t] + j];
            }
#pragma unroll
            for (uint32_t t = 0; t < (uint32_t)NP; t++) {
                const bool up = (ii[t] & k) == 0u;
                if (up ? x[t] > y[t] : x[t] < y[t]) {
                    v[ii[t]] = y[t];
                    v[ii[t] + j] = x[t];
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
}

// Runs of a key of more than kRoBucket runs, in position order, for its walk wave: the
// bucket (bv, one run per lane) and the placed overflow runs (index >= kRoBucket), padded to
// a power of two and sorted by start -- up to kRoSortLds runs by a bitonic wave sort in the
// wave's LDS region, else in its region of sortTmp (at twice the
// key's place, so regions of different keys never meet) through agent-scope loads and
// stores, which every lane of the wave sees after the stage's vmcnt(0).  Returns where the
// sorted runs are.
__device__ unsigned long long *ro_sort_runs(const RoScratch &sc, uint32_t slot, uint32_t c, unsigned long long bv,
                                            unsigned long long *lds, uint32_t lane)
{
    const uint32_t rb = sc.runBase[slot];
    const unsigned long long *ov = sc.placed + rb;
    uint32_t P = 64;
    while (P < c) P <<= 1;
    if (P <= kRoSortLds) {
        for (uint32_t i = lane; i < P; i += 64u) lds[i] = i < kRoBucket ? bv : (i < c ? ov[i] : ~0ull);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (P <= 128u) wave_sort_lds<1>(lds, lane);
        else if (P <= 256u) wave_sort_lds<2>(lds, lane);
        else if (P <= 512u) wave_sort_lds<4>(lds, lane);
        else if (P <= 1024u) wave_sort_lds<8>(lds, lane);
        else wave_sort_lds<16>(lds, lane);
        return lds;
    }
    unsigned long long *g = sc.sortTmp + 2ull * rb;
    for (uint32_t i = lane; i < P; i += 64u)
        __hip_atomic_store(g + i, i < kRoBucket ? bv : (i < c ? ov[i] : ~0ull), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (uint32_t k = 2; k <= P; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = lane; i < P; i += 64u) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const unsigned long long x = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const unsigned long long y = __hip_atomic_load(g + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (((i & k) == 0u) ? x > y : x < y) {
                        __hip_atomic_store(g + i, y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(g + l, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    return g;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v)
{
#pragma unroll
    for (int o = 32; o; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
#pragma unroll
    for (int o = 32; o; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}

// The positions of a key of more than kRoBucket runs, in arrival order, into the wave's LDS
// region, without sorting its runs: every run sets its positions' bits in a bitmap over the
// key's span (LDS atomic ORs), and the set bits read in order are the positions.  Returns
// how many (0 when bitmap and list do not fit the region: then the runs are sorted).
__device__ uint32_t ro_positions(const RoScratch &sc, uint32_t slot, uint32_t c, unsigned long long bv,
                                 unsigned long long *lds, uint32_t lane, uint32_t ldsWords)
{
    const unsigned long long *ov = sc.placed + sc.runBase[slot];
    uint32_t mn = 0xFFFFFFFFu, mx = 0, tl = 0;
    for (uint32_t i = lane; i < c; i += 64u) {
        const unsigned long long r = i < kRoBucket ? bv : ov[i];
        const uint32_t st = (uint32_t)(r >> 32), ln = (uint32_t)r;
        mn = min(mn, st);
        mx = max(mx, st + ln);
        tl += ln;
    }
    mn = wave_min_u32(mn);
    mx = wave_max_u32(mx);
    tl = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(tl), 63);
    const uint32_t words = (mx - mn + 63u) / 64u;
    if ((size_t)words * 8u + (size_t)tl * 4u > (size_t)ldsWords * 8u) return 0u;     // wave-uniform
    for (uint32_t i = lane; i < words; i += 64u) lds[i] = 0ull;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t i = lane; i < c; i += 64u) {
        const unsigned long long r = i < kRoBucket ? bv : ov[i];
        const uint32_t b = (uint32_t)(r >> 32) - mn, ln = (uint32_t)r;   // 1..64 positions
        const unsigned long long m = ln >= 64u ? ~0ull : ((1ull << ln) - 1ull);
        const uint32_t o = b & 63u;
        atomicOr(&lds[b >> 6], m << o);
        if (o + ln > 64u) atomicOr(&lds[(b >> 6) + 1u], m >> (64u - o));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // each lane reads a contiguous block of words; a wave scan of their counts places them
    const uint32_t wpl = (words + 63u) / 64u, w0 = lane * wpl, w1 = min(w0 + wpl, words);
    uint32_t cnt = 0;
    for (uint32_t x = w0; x < w1; x++) cnt += (uint32_t)__builtin_popcountll(lds[x]);
    uint32_t at = wave_incl_scan(cnt) - cnt;
    uint32_t *pos = reinterpret_cast<uint32_t *>(lds + words);
    for (uint32_t x = w0; x < w1; x++)
        for (unsigned long long m = lds[x]; m; m &= m - 1ull) pos[at++] = mn + x * 64u + (uint32_t)__builtin_ctzll(m);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the list starts at lds + words: move it to the front (the walk reads it from there)
    uint32_t *dst = reinterpret_cast<uint32_t *>(lds);
    for (uint32_t i = lane; i < tl; i += 64u) {
        const uint32_t v = pos[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        dst[i] = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return tl;
}

// WB waves per workgroup, LW 8-byte words of LDS per wave (the position bitmap and list, or
// the LDS sort of <= kRoSortLds runs)
template <int WB, uint32_t LW>
__global__ __launch_bounds__(WB * 64) void ro_walk_kernel(ReasDev R, RoScratch sc, uint32_t T, uint64_t now,
                                                          PktInfo *__restrict__ info, FinishRec *__restrict__ fin)
{
    static_assert(LW >= kRoSortLds, "the LDS sort needs kRoSortLds words");
    __shared__ unsigned long long roSort[WB][LW];
    const uint32_t w = blockIdx.x * (uint32_t)WB + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    // the chain of dependent loads before the walk proper is kept short: the key is read
    // beside the count of keys, and its bucket beside its run count
    const uint32_t nKeys = sc.ctr[2];
    const uint32_t slot = w < T ? sc.active[w] : 0u;
    if (w >= nKeys) return;                                    // wave-uniform
    const uint32_t nRuns = sc.runCnt[slot];
    const unsigned long long bv = sc.bucket[(size_t)slot * kRoBucket + lane];
    const bool inBucket = nRuns <= kRoBucket;
    if (w == 0 && lane == 0) sc.ctr[0] = 0u;                   // overflow runs: next batch
    unsigned long long *lds = roSort[threadIdx.x >> 6];
    const unsigned long long *runsOf = nullptr;
    uint32_t nPos = 0;                                         // > 0: the key's positions are in lds
    if (!inBucket) {
        nPos = ro_positions(sc, slot, nRuns, bv, lds, lane, LW);
        if (nPos == 0u) runsOf = ro_sort_runs(sc, slot, nRuns, bv, lds, lane);
    }
    const RoRec *__restrict__ recs = sc.recs;
    ReasSlot *sl = R.slots + slot;
    const uint64_t ev = sl->eventNum;
    const uint32_t d = sl->dataId;
    bool item = sl->bvalid == 1u;                              // an item in progress from an earlier batch
    uint64_t boff = sl->bufOff;
    uint32_t ibytes = sl->bytes;
    uint64_t cur = item ? (sl->acc & kAccBytesMask) : 0ull;
    uint32_t frags = item ? (uint32_t)(sl->acc >> kAccFragShift) : 0u;
    uint64_t created = sl->created;
    long long live = 0;                                        // net change of items in progress
    uint32_t derr = 0;
    uint32_t tot = 0;                                          // datagrams of the current walk
    // one chunk of 64 datagrams of the key, in arrival order (q: position, rc: record)
    auto walk_chunk = [&](uint32_t base, uint32_t q, const RoRec &rc) {
        const bool valid = base + lane < tot;
        const uint32_t nv = (tot - base < 64u) ? tot - base : 64u;
        for (uint32_t t = 0; t < nv;) {
            if (!item || (uint32_t)__builtin_amdgcn_readlane((int)rc.off, (int)t) == 0u) {
                // a new item (EventQueueItem(rehdr), hpp:89-98); at offset 0 it replaces the
                // one in progress (cpp:361-369), dropped without a lost record
                if (item) live--;
                const uint32_t blen = (uint32_t)__builtin_amdgcn_readlane((int)rc.blen, (int)t);
                const uint64_t need = ((uint64_t)blen + 255ull) & ~255ull;
                uint64_t nb = 0;
                if (lane == 0) nb = atomicAdd(&R.ctl->arenaTop, (unsigned long long)(need ? need : 256ull));
                nb = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(nb >> 32), 0) << 32) |
                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)nb, 0);
                if (nb + blen > R.arenaBytes) {
                    if (lane == 0) atomicOr(&R.ctl->errorFlags, 2u);
                    nb = kNoBuf;
                }
                boff = nb;
                ibytes = blen;
                cur = 0;
                frags = 0;
                created = now;
                item = true;
                live++;
            }
            const uint64_t zm = __ballot(valid && rc.off == 0u && lane > t);
            const uint32_t v = zm ? (uint32_t)__builtin_ctzll(zm) : nv;      // next item start
            const bool inseg = lane >= t && lane < v;
            const bool viol = inseg && (uint64_t)rc.off + rc.plen > ibytes;
            const uint32_t P = wave_incl_scan((inseg && !viol) ? rc.plen : 0u);
            const uint64_t cm = __ballot(inseg && !viol && cur + P == (uint64_t)ibytes);
            const uint32_t end = cm ? (uint32_t)__builtin_ctzll(cm) + 1u : v;
            const bool inr = lane >= t && lane < end;
            frags += (uint32_t)__builtin_popcountll(__ballot(inr && !viol));     // cpp:398-400
            derr += (uint32_t)__builtin_popcountll(__ballot(inr && viol));
            cur += (uint32_t)__builtin_amdgcn_readlane((int)P, (int)(end - 1u));
            const bool comp = cm && lane == end - 1u;
            if (inr) {
                PktInfo pi{0ull, 0u, rc.hl};
                if (!viol && boff != kNoBuf) {
                    pi.dst = (uint64_t)(R.arena + boff + rc.off);
                    pi.plen = rc.plen;
                }
                if (comp) {                                    // cpp:403: complete, erase, enqueue
                    FinishRec f;
                    f.ev = ev;
                    f.boff = boff;
                    f.slot = slot | kFinKeepSlot;
                    f.bytes = ibytes;
                    f.frags = frags;
                    f.d = d;
                    fin[q] = f;
                    pi.hl |= kPktCompletes;
                }
                st16(reinterpret_cast<uint8_t *>(info + q), u32x4{(uint32_t)pi.dst, (uint32_t)(pi.dst >> 32), pi.plen, pi.hl});
            }
            if (cm) item = false;                              // inProgress-- in complete_event
            t = end;
        }
    };
    // the records of the next kRoAhead - 1 chunks are in flight while a chunk is walked (the
    // walk is a chain of dependent chunks over few waves: latency, not bandwidth, bounds it).
    // The ring is indexed statically (unrolled by kRoAhead); a chunk's slot is reloaded after
    // the chunk is walked.  (Round 5: staging a key's records in LDS by LDS-DMA, 16 chunks per
    // wait, measured 16.6 against this ring's 15.5 us per launch: the chunks' own work, ~0.8
    // us each at one wave per CU, not their loads, bounds the walk)
    auto walk_ring = [&](auto q_of) {
    uint32_t qr[kRoAhead];
    RoRec rr[kRoAhead];
#pragma unroll
    for (uint32_t i = 0; i < kRoAhead; i++) {
        qr[i] = q_of(i * 64u);
        rr[i] = RoRec{0u, 0u, 0u, 0u};
        if (i * 64u + lane < tot) rr[i] = recs[qr[i]];
    }
    for (uint32_t b0 = 0; b0 < tot; b0 += kRoAhead * 64u) {
#pragma unroll
        for (uint32_t i = 0; i < kRoAhead; i++) {
            const uint32_t base = b0 + i * 64u;
            if (base < tot) {                                  // wave-uniform
                walk_chunk(base, qr[i], rr[i]);
                const uint32_t nxt = base + kRoAhead * 64u;
                if (nxt < tot) {
                    qr[i] = q_of(nxt);
                    if (nxt + lane < tot) rr[i] = recs[qr[i]];
                }
            }
        }
    }
    };
    if (nPos) {
        // the key's positions in arrival order, from its position bitmap
        const uint32_t *pos = reinterpret_cast<const uint32_t *>(lds);
        tot = nPos;
        walk_ring([&](uint32_t base) -> uint32_t { return base + lane < tot ? pos[base + lane] : 0u; });
    } else {
    for (uint32_t r0 = 0; r0 < nRuns; r0 += 64u) {
    // this batch of the key's runs, in position order: start << 32 | length per lane
    const uint32_t m = (nRuns - r0 < 64u) ? nRuns - r0 : 64u;
    unsigned long long rv = (lane < m) ? (inBucket ? bv : runsOf[r0 + lane]) : ~0ull;
    if (inBucket) {
        // order the bucket by start (the starts are distinct): each run's rank is the number
        // of runs that start before it (m scalar reads), then one push per word to lane rank
        const uint32_t mys = (uint32_t)(rv >> 32);
        uint32_t rank = 0;
        for (uint32_t r = 0; r < m; r++) rank += (uint32_t)__builtin_amdgcn_readlane((int)mys, (int)r) < mys ? 1u : 0u;
        if (lane >= m) rank = lane;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_permute((int)(rank * 4u), (int)(uint32_t)rv);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_permute((int)(rank * 4u), (int)mys);
        rv = ((unsigned long long)hi << 32) | lo;
    }
    const uint32_t rlen = (uint32_t)rv & 0xFFFFFFFFu, rstart = (uint32_t)(rv >> 32);
    const uint32_t rl = lane < m ? rlen : 0u;
    const uint32_t rin = wave_incl_scan(rl), rex = rin - rl;
    tot = (uint32_t)__builtin_amdgcn_readlane((int)rin, 63);
    // position of datagram base + lane of this batch of runs: in the last run whose prefix
    // is <= it.  The runs that meet the chunk [base, base + 64) are r0..r1 (usually two): a
    // uniform loop over them with scalar reads, no per-lane search
    auto pos_of = [&](uint32_t base) -> uint32_t {
        const uint32_t g = base + lane;
        const uint64_t b0 = __ballot(lane < m && rex <= base), b1 = __ballot(lane < m && rex < base + 64u);
        const int r0 = b0 ? 63 - __builtin_clzll(b0) : 0, r1 = b1 ? 63 - __builtin_clzll(b1) : 0;
        uint32_t qb = 0;
        for (int r = r0; r <= r1; r++) {
            const uint32_t sr = (uint32_t)__builtin_amdgcn_readlane((int)rex, r);
            const uint32_t st = (uint32_t)__builtin_amdgcn_readlane((int)rstart, r);
            if (g >= sr) qb = st - sr;
        }
        return qb + g;
    };
    walk_ring(pos_of);
    }
    }
    if (lane == 0) {
        sc.runCnt[slot] = 0u;                                  // next batch
        if (item) {
            sl->bufOff = boff;
            sl->bytes = ibytes;
            sl->bvalid = 1u;
            sl->acc = ((unsigned long long)frags << kAccFragShift) | (cur & kAccBytesMask);
            sl->created = created;
        } else {
            sl->state = kDone;                                 // no item left under this key
        }
        if (live) atomicAdd(occ_in_progress(R, slot), (unsigned long long)live);
        if (derr) atomicAdd(&R.shards[slot % kShards].dataErrCnt, (unsigned long long)derr);
    }
}

// Zero nWords dwords.  Used instead of hipMemsetAsync wherever the launch may be captured
// into a HIP graph: on this ROCm captured hipMemsetAsync nodes write garbage from the
// second replay on (fill_bytes_kernel below).
__global__ __launch_bounds__(kBlock) void zero_words_kernel(uint32_t *p, uint64_t nWords)
{
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nWords; i += (uint64_t)gridDim.x * kBlock)
        p[i] = 0u;
}

// Fill bytes [p, p + n) with v: bytes up to the first 16-byte boundary and after the last,
// 16-byte stores in between.  e2sar_hip_memset_d uses it instead of hipMemsetAsync: on this
// ROCm a captured hipMemsetAsync node of 64 bytes or more writes garbage from the second
// graph replay on (tools/graph_memset_probe.py); a kernel node replays clean.
__global__ __launch_bounds__(kBlock) void fill_bytes_kernel(uint8_t *p, uint8_t v, uint64_t n)
{
    const uint64_t head = ((16u - ((uintptr_t)p & 15u)) & 15u) < n ? ((16u - ((uintptr_t)p & 15u)) & 15u) : n;
    const uint64_t body = (n - head) & ~15ull;
    const uint64_t t0 = (uint64_t)blockIdx.x * kBlock + threadIdx.x, step = (uint64_t)gridDim.x * kBlock;
    if (t0 < head) st1(p + t0, v);
    const uint64_t tail0 = head + body;
    if (t0 < n - tail0) st1(p + tail0 + t0, v);
    const uint32_t w = 0x01010101u * v;
    const u32x4 q{w, w, w, w};
    for (uint64_t i = t0; i < body / 16u; i += step) st16(p + head + 16u * i, q);
}

hipError_t launch_fill_bytes(void *p, int value, uint64_t n, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n / 16u + kBlock - 1u) / kBlock + 1u;
    hipLaunchKernelGGL(fill_bytes_kernel, dim3((uint32_t)(blocks < 4096 ? blocks : 4096)), dim3(kBlock), 0, stream,
                       static_cast<uint8_t *>(p), (uint8_t)value, n);
    return hipGetLastError();
}

// Gather copy: blockIdx.y = span; 16-byte loads and stores when both ends are 16-byte
// aligned (arena event buffers are 256-aligned; callers lay destinations out 64-aligned),
// bytes otherwise and for the tail.
// One workgroup copies one 8-KiB piece of one span (blockIdx.y): every thread issues its
// two 16-byte non-temporal loads before any store, as seg_kernel does, so a large span
// streams at the plain-copy rate (the bench's HBM calibration copies 1 and 4 GiB with it).
// 8-KiB pieces copy faster than 16-KiB ones on random bytes (tools/ubench_store.hip:
// 6.06 vs 5.99 TB/s at 1 GiB, 6.21 vs 5.99 at 4 GiB).
constexpr int kCopyU = 2;
constexpr uint32_t kCopyPiece = (uint32_t)kBlock * 16u * kCopyU;
__global__ __launch_bounds__(kBlock) void copy_spans_kernel(CopySpans cs)
{
    if (blockIdx.y >= cs.n) return;
    const CopySpan sp = cs.s[blockIdx.y];
    const uint64_t base = (uint64_t)blockIdx.x * kCopyPiece;
    if (base >= sp.bytes) return;
    const uint8_t *src = reinterpret_cast<const uint8_t *>(sp.src);
    uint8_t *dst = reinterpret_cast<uint8_t *>(sp.dst);
    const uint64_t end = (base + kCopyPiece < sp.bytes) ? base + kCopyPiece : sp.bytes;
    uint64_t b0 = base;
    if (((sp.src | sp.dst) & 15u) == 0) {
        const uint64_t whole = sp.bytes & ~15ull;
        u32x4 x[kCopyU];
#pragma unroll
        for (int u = 0; u < kCopyU; u++) {
            const uint64_t i = base + 16ull * ((uint64_t)u * kBlock + threadIdx.x);
            x[u] = (i + 16 <= whole) ? ld16_nt(src + i) : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int u = 0; u < kCopyU; u++) {
            const uint64_t i = base + 16ull * ((uint64_t)u * kBlock + threadIdx.x);
            if (i + 16 <= whole) st16_nt(dst + i, x[u]);
        }
        b0 = (whole > base) ? ((whole < end) ? whole : end) : base;
    }
    for (uint64_t b = b0 + threadIdx.x; b < end; b += kBlock) dst[b] = src[b];
}

hipError_t launch_copy_spans(const CopySpans &cs, uint64_t largest, hipStream_t stream)
{
    if (cs.n == 0 || largest == 0) return hipSuccess;
    const uint64_t bx = (largest + kCopyPiece - 1) / kCopyPiece;
    if (bx > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(copy_spans_kernel, dim3((uint32_t)bx, cs.n), dim3(kBlock), 0, stream, cs);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// GC / recycle

__global__ __launch_bounds__(kBlock) void reas_gc_kernel(ReasDev R, uint64_t now, uint64_t timeout)
{
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= R.tableSlots) return;
    ReasSlot *sl = R.slots + s;
    if (ld_agent(&sl->state) != kReady) return;
    const uint64_t created = ld_agent(&sl->created);
    if (now <= created || now - created <= timeout) return;     // inWaiting > timeout (cpp:262)
    if (atomicCAS(&sl->state, (uint32_t)kReady, (uint32_t)kLost) != kReady) return;
    atomicAdd(&R.ctl->reassemblyLoss, 1ull);
    atomicAdd(occ_in_progress(R, s), ~0ull);
    const uint32_t li = atomicAdd(&R.ctl->nLost, 1u);
    if (li < R.lostCapacity) {
        e2sar_hip_lost_rec rec;
        rec.eventNum = ld_agent(&sl->eventNum);
        rec.numFragments = ld_agent(&sl->acc) >> kAccFragShift;
        rec.dataId = (uint16_t)ld_agent(&sl->dataId);
        rec.enqueueLoss = 0;
        rec.reserved = 0;
        R.lost[li] = rec;
    }
}

__device__ void recycle_slots(const ReasDev &R, uint32_t s, int dropCompleted)
{
    if (s < R.tableSlots) {
        ReasSlot z{};
        R.slots[s] = z;
    }
    if (s == 0) {
        R.ctl->arenaTop = 0;
        R.ctl->tableUsed = 0;
        R.ctl->inProgress = 0;
        if (dropCompleted) R.ctl->nCompleted = 0;
    }
    if (s < kShards) {
        *occ_in_progress(R, s) = 0ull;
        *occ_table_used(R, s) = 0ull;
    }
}

__global__ __launch_bounds__(kBlock) void reas_recycle_kernel(ReasDev R, int dropCompleted)
{
    recycle_slots(R, blockIdx.x * kBlock + threadIdx.x, dropCompleted);
}

// Compaction: one block per slot of `from`.  Surviving (READY) events get a new buffer
// at the bottom of the `to` arena and a slot in the (empty) `to` table; their partial
// bytes are copied whole.  Nothing else touches either table during this launch, so the
// insert needs only the CAS for slot ownership among compacting blocks.
__global__ __launch_bounds__(kBlock) void reas_compact_kernel(ReasDev from, ReasDev to)
{
    __shared__ uint64_t sOff;
    const ReasSlot *sl = from.slots + blockIdx.x;
    if (sl->state != kReady) return;
    const uint32_t bytes = sl->bytes;
    if (threadIdx.x == 0) {
        uint64_t off = kNoBuf;
        if (sl->bufOff != kNoBuf) {
            const uint64_t need = ((uint64_t)bytes + 255ull) & ~255ull;
            off = atomicAdd(&to.ctl->compactTop, (unsigned long long)(need ? need : 256ull));
            if (off + bytes > to.arenaBytes) {
                off = kNoBuf;                      // cannot happen when to.arenaBytes >= from.arenaBytes
                atomicOr(&to.ctl->errorFlags, 2u);
            }
        }
        const uint32_t mask = to.tableSlots - 1u;
        uint32_t h = slot_hash(sl->eventNum, sl->dataId, mask);
        for (uint32_t probe = 0; probe < to.tableSlots; probe++, h = (h + 1u) & mask) {
            if (atomicCAS(&to.slots[h].state, (uint32_t)kEmpty, (uint32_t)kBusy) == kEmpty) {
                ReasSlot *d = to.slots + h;
                d->dataId = sl->dataId;
                d->bytes = bytes;
                d->eventNum = sl->eventNum;
                d->acc = sl->acc;
                d->bufOff = off;
                d->bvalid = 1u;
                d->created = sl->created;
                d->state = kReady;
                atomicAdd(&to.ctl->compactUsed, 1u);
                break;
            }
        }
        sOff = off;
    }
    __syncthreads();
    const uint64_t off = sOff;
    if (off == kNoBuf || sl->bufOff == kNoBuf) return;
    const uint8_t *src = from.arena + sl->bufOff;
    uint8_t *dst = to.arena + off;
    const uint32_t n16 = bytes >> 4;
    for (uint32_t i = threadIdx.x; i < n16; i += kBlock) st16(dst + 16u * i, ld16(src + 16u * i));
    for (uint32_t b = (n16 << 4) + threadIdx.x; b < bytes; b += kBlock) st1(dst + b, ld1(src + b));
}

__global__ void reas_compact_finish(ReasDev to)
{
    to.ctl->arenaTop = to.ctl->compactTop;
    to.ctl->tableUsed = to.ctl->compactUsed;
    for (uint32_t k = 0; k < kShards; k++) *occ_table_used(to, k) = 0ull;
    to.ctl->compactTop = 0;
    to.ctl->compactUsed = 0;
}

// ---------------------------------------------------------------------------------
// launchers

static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

hipError_t launch_zero_words(void *p, uint64_t nWords, hipStream_t stream)
{
    if (nWords == 0) return hipSuccess;
    const uint64_t blocks = (nWords + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(zero_words_kernel, dim3((uint32_t)(blocks < 4096 ? blocks : 4096)), dim3(kBlock), 0, stream,
                       static_cast<uint32_t *>(p), nWords);
    return hipGetLastError();
}

// Occupancy caps by dynamic LDS: the dynamic LDS that holds a launch of `kernel` (its own
// static LDS included) to at most perCU workgroups per CU on the current device, from the
// device's LDS per CU and per workgroup -- 0 (no cap) where the cap cannot be expressed.
// The caps were measured on gfx950 (160 KiB of LDS per CU); computed here, they mean the
// same workgroups per CU on any LDS size instead of a fixed byte count.
template <typename K>
static size_t occupancy_lds(K kernel, uint32_t perCU)
{
    static std::atomic<int> ldsCU[64], ldsWG[64];
    int dev = 0;
    if (perCU == 0 || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    int cu = ldsCU[dev].load(std::memory_order_relaxed), wg = ldsWG[dev].load(std::memory_order_relaxed);
    if (cu <= 0 || wg <= 0) {
        if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess ||
            hipDeviceGetAttribute(&wg, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || cu <= 0 || wg <= 0) {
            (void)hipGetLastError();
            return 0;
        }
        ldsCU[dev].store(cu, std::memory_order_relaxed);
        ldsWG[dev].store(wg, std::memory_order_relaxed);
    }
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(kernel)) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    size_t T = ((size_t)cu / perCU) & ~(size_t)1023;                  // bytes per workgroup
    if (T > (size_t)wg) T = (size_t)wg;
    if (T <= fa.sharedSizeBytes || (size_t)cu / T != perCU) return 0;  // perCU fit, perCU + 1 do not
    return T - fa.sharedSizeBytes;
}

template <int U, int NT>
static uint32_t reas_resident_groups();

// Geometry of seg_kernel for a batch: 16-byte chunks per thread, units per event and the
// XCD stripe (units per stripe, 0 = none).  One place, so the reassembly group table of
// seg_groups always matches the launch.
struct SegGeom {
    uint32_t U, unitChunks, bpe, stripe;
    uint64_t nUnits;
};
static bool seg_geom(uint32_t nEvents, uint32_t maxPacketsPerEvent, uint32_t stride, SegGeom &g)
{
    const uint32_t spc = stride >> 4;
    const uint64_t chunks = (uint64_t)maxPacketsPerEvent * spc;
    if (chunks > 0xFFFFFFFFull || spc == 0) return false;        // chunk index of an event is u32
    g.U = chunks <= (1u << 18) ? 2u : 4u;
    g.unitChunks = (uint32_t)kSegBlock * g.U;
    g.bpe = cdiv(chunks, g.unitChunks);
    g.nUnits = (uint64_t)g.bpe * nEvents;
    // a stripe of about one fused reassembly group, min(49, 9216 / spc) datagrams, then
    // balanced as reas_group_size balances its groups: the stripe count (= reassembly
    // workgroups) just under a whole number of the chip's residency waves, if that keeps
    // the stripe within [3/4, 4/3] of the target (205 x 1 MiB at MTU 1500: 8 -> 9 units,
    // 3383 -> 3007 groups for 2 x 1536 resident)
    g.stripe = 0;
    const uint32_t target = std::min<uint32_t>(49u, std::max<uint32_t>(1u, kReasChunksPerBlock / spc));
    const uint32_t S0 = std::max<uint32_t>(1u, (uint32_t)((uint64_t)target * spc / g.unitChunks));
    uint32_t best = S0;
    const uint32_t cap = reas_resident_groups<kReasU, kBlock>();
    if (cap && g.nUnits) {
        const uint64_t waves = ((g.nUnits + S0 - 1) / S0 + cap - 1) / cap;
        uint32_t bestDev = ~0u;
        for (uint64_t k = (waves > 1 ? waves - 1 : waves); k <= waves; k++) {
            const uint64_t c = (g.nUnits + k * cap - 1) / (k * cap);
            if (c == 0 || c > 0xFFFFu || 4u * c < 3u * S0 || 3u * c > 4u * S0) continue;
            const uint32_t dev = (uint32_t)(c > S0 ? c - S0 : S0 - c);
            if (dev < bestDev) best = (uint32_t)c, bestDev = dev;
        }
    }
    g.stripe = best;
    return true;
}

hipError_t launch_segment(const e2sar_hip_seg_event *d_events, uint32_t nEvents,
                          uint32_t maxPacketsPerEvent, int lbVersion, uint32_t maxPld,
                          uint8_t *pkts, uint32_t stride, uint32_t *lens,
                          hipStream_t stream, const uint32_t *d_count, const ReasDev *rec, bool dropCompleted)
{
    if (nEvents == 0 || maxPacketsPerEvent == 0) return rec ? launch_recycle(*rec, dropCompleted, stream) : hipSuccess;
    SegGeom sg;
    if (!seg_geom(nEvents, maxPacketsPerEvent, stride, sg)) return hipErrorInvalidValue;
    const uint64_t segGrid = sg.stripe ? (sg.nUnits + 8ull * sg.stripe - 1) / (8ull * sg.stripe) * 8ull * sg.stripe
                                       : sg.nUnits;
    const uint64_t grid = segGrid + (rec ? cdiv(rec->tableSlots > kShards ? rec->tableSlots : (uint32_t)kShards,
                                                (uint32_t)kSegBlock) : 0u);
    if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
    const ReasDev none{};
    const ReasDev &rj = rec ? *rec : none;
    const int mode = rec ? (dropCompleted ? 2 : 1) : 0;
    if (sg.U == 2)
        hipLaunchKernelGGL((seg_kernel<2>), dim3((uint32_t)grid), dim3(kSegBlock), 0, stream, d_events,
                           sg.bpe, lbVersion, maxPld, pkts, stride, lens, d_count, sg.stripe, (uint32_t)sg.nUnits, rj,
                           (uint32_t)segGrid, mode);
    else
        hipLaunchKernelGGL((seg_kernel<4>), dim3((uint32_t)grid), dim3(kSegBlock), occupancy_lds(seg_kernel<4>, kSeg4PerCU),
                           stream, d_events, sg.bpe, lbVersion, maxPld, pkts, stride, lens, d_count, sg.stripe,
                           (uint32_t)sg.nUnits, rj, (uint32_t)segGrid, mode);
    return hipGetLastError();
}

// Reassembly groups that match seg_kernel's XCD stripes for a planned batch (host event
// table with pktBase, as e2sar_hip_seg_plan fills it): group m = the datagrams whose first
// chunk lies in stripe m (units [m * stripe, (m + 1) * stripe)), written on XCD m mod 8;
// reas_kernel workgroup m runs on the same XCD.  starts[0..nGroups], nGroups + 1 <= cap.
// Returns nGroups, or 0 when the batch has no stripes or a group would exceed 64
// datagrams (the caller then reassembles with the uniform groups).
uint32_t seg_groups(const e2sar_hip_seg_event *ev, uint32_t nEvents, uint32_t maxPacketsPerEvent, uint32_t maxPld,
                    uint32_t stride, uint32_t *starts, uint32_t cap)
{
    SegGeom sg;
    if (nEvents == 0 || maxPld == 0 || !seg_geom(nEvents, maxPacketsPerEvent, stride, sg) || !sg.stripe) return 0;
    const uint64_t nGroups = (sg.nUnits + sg.stripe - 1) / sg.stripe;
    if (nGroups + 1 > cap || nGroups > 0x7FFFFFFFull) return 0;
    const uint32_t spc = stride >> 4;
    uint64_t g = 0, total = 0;
    starts[0] = 0;
    for (uint32_t e = 0; e < nEvents; e++) {
        const uint32_t np = (uint32_t)(((uint64_t)ev[e].bytes + maxPld - 1u) / maxPld);   // 0 for an empty event
        const uint32_t base = ev[e].pktBase;
        for (uint32_t q = 0; q < np; q++) {
            const uint64_t m = ((uint64_t)e * sg.bpe + (uint64_t)q * spc / sg.unitChunks) / sg.stripe;
            while (g < m) {
                starts[++g] = base + q;
                if (starts[g] - starts[g - 1] > 64u) return 0;
            }
        }
        total = (uint64_t)base + np;
    }
    while (g < nGroups) {
        starts[++g] = (uint32_t)total;
        if (starts[g] - starts[g - 1] > 64u) return 0;
    }
    return (uint32_t)nGroups;
}

// ---------------------------------------------------------------------------------
// relay: the events a reassembler completed become a segmentation batch on the device
//
// One workgroup reads completed records [first, first + n) (n = min(maxEvents, records
// stored - first)), writes one seg descriptor per event -- the event's arena bytes, its RE
// eventNum and dataId as received, the batch's LB tick, entropy entropyBase + i -- with
// pktBase the exclusive prefix of ceil(bytes / maxPld) (a block-wide scan, 256 records per
// step), and counts[0] = n, counts[1] = the batch's datagram count.

__global__ __launch_bounds__(kBlock) void relay_plan_kernel(ReasDev R, uint32_t first, uint32_t maxEvents,
                                                            uint32_t maxPld, uint64_t lbTick, uint32_t entropyBase,
                                                            e2sar_hip_seg_event *__restrict__ out,
                                                            uint32_t *__restrict__ counts)
{
    __shared__ uint32_t waveSum[kBlock / 64];
    __shared__ uint32_t sN;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        uint32_t stored = ld_agent(&R.ctl->nCompleted);
        if (stored > R.queueCapacity) stored = R.queueCapacity;        // records past it were lost
        const uint32_t avail = stored > first ? stored - first : 0u;
        sN = avail < maxEvents ? avail : maxEvents;
    }
    __syncthreads();
    const uint32_t n = sN;
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < n; b0 += kBlock) {
        const uint32_t i = b0 + threadIdx.x;
        e2sar_hip_event_rec rec{};
        if (i < n) rec = R.completed[first + i];
        const uint32_t np = (i < n) ? (rec.bytes + maxPld - 1u) / maxPld : 0u;
        uint32_t inc = np;                                   // inclusive scan in the wave
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
        }
        if (lane == 63) waveSum[wv] = inc;
        __syncthreads();
        uint32_t before = carry;
        for (uint32_t w = 0; w < wv; w++) before += waveSum[w];
        if (i < n) {
            e2sar_hip_seg_event d;
            d.data = R.arena + rec.arenaOffset;
            d.eventNum = rec.eventNum;
            d.lbTick = lbTick;
            d.bytes = rec.bytes;
            d.pktBase = before + inc - np;
            d.dataId = rec.dataId;
            d.entropy = (uint16_t)(entropyBase + i);
            d.reserved = 0;
            out[i] = d;
        }
        for (uint32_t w = 0; w < kBlock / 64; w++) carry += waveSum[w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        counts[0] = n;
        counts[1] = carry;
    }
}

hipError_t launch_relay_plan(const ReasDev &R, uint32_t first, uint32_t maxEvents, uint32_t maxPld,
                             uint64_t lbTick, uint32_t entropyBase, e2sar_hip_seg_event *d_events,
                             uint32_t *d_counts, hipStream_t stream)
{
    hipLaunchKernelGGL(relay_plan_kernel, dim3(1), dim3(kBlock), 0, stream, R, first, maxEvents, maxPld, lbTick,
                       entropyBase, d_events, d_counts);
    return hipGetLastError();
}

// Where the pipelined launch's classify workgroups sit, percent of the way through its
// scatter workgroups (launch_reas_scatter_classify)
constexpr uint32_t kPipeClsAtPercent = 75;

// Scatter workgroups of the launch: groups of G whole datagrams; returns G and the
// workgroup count.
__host__ __device__ constexpr int scatter_u(uint32_t stride) { return stride > 4096u ? kScatUJumbo : kScatU; }
__host__ __device__ constexpr int scatter_tb(uint32_t stride) { return stride > 4096u ? kScatBlockJumbo : kScatBlock; }
static uint32_t scatter_group_size(uint32_t stride)
{
    // datagrams per scatter workgroup: at most one round of 16-byte chunks (256 threads x
    // scatter_u), <= 64.  The scatter needs no table round trip, so it
    // streams best in one-round workgroups, like seg_kernel: at 205 x 1 MiB, MTU 1500, a
    // batch read back cold takes 81.5 us with 1K-chunk groups against 100.3 us with the
    // fused kernel's 9K budget (89.5 us at 2K); hot, 68.7 us.
    const uint32_t spc = stride >> 4;
    uint32_t G = 64;
    while (G > 1 && G * spc > (uint32_t)(scatter_tb(stride) * scatter_u(stride))) G >>= 1;
    return G;
}
static uint32_t scatter_geometry(uint32_t stride, uint32_t n, uint32_t &blocks)
{
    const uint32_t G = scatter_group_size(stride);
    blocks = cdiv(n, G);
    return G;
}

// Workgroups of reas_kernel<U, NT> the current device holds at once (0 if unknown), per device.
template <int U, int NT>
static uint32_t reas_resident_groups()
{
    static std::atomic<uint32_t> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    uint32_t c = cache[dev].load(std::memory_order_relaxed);
    if (c) return c;
    int per = 0, cus = 0;
    // the uncapped occupancy, as the jumbo launch's cap was measured (balancing on the
    // capped one tied, profiles/round4/ab/reas_small_caps.log)
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reas_kernel<U, NT>, NT, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per <= 0 || cus <= 0)
        return 0;
    c = (uint32_t)per * (uint32_t)cus;
    cache[dev].store(c, std::memory_order_relaxed);
    return c;
}

// fixedG: the reassembler's configured group size (e2sar_hip_reas_config.groupSize), 0 = auto
static uint32_t reas_group_size(uint32_t n, uint32_t stride, uint32_t fixedG, int NT)
{
    if (fixedG) return fixedG < 64u ? fixedG : 64u;
    constexpr int U = kReasU;
    // datagrams per workgroup: at most kReasChunksPerBlock 16-byte chunks, <= 64.
    // (A/B: at MTU 1500 2K-chunk groups lose ~8 %, 1K ~30 %, 4K-12K equal; at MTU 9000 with
    // 8 MiB events 4K chunks (4 datagrams per group) lose 27 % to 9K-18K: per-event counter
    // and table traffic grows with groups per event)
    const uint32_t spc = stride >> 4, budget = kReasChunksPerBlock;
    uint32_t G = 64;
    while (G > 1 && G * spc > budget) G >>= 1;
    // Balance the launch over whole residency waves: with ceil(n/G) workgroups = 1.5 x
    // what the chip holds at once, the second wave starts late and the last ~15 us run
    // half-empty (tools/trace_reas.py). Pick G so the workgroup count is just under a
    // whole number of waves -- one wave more (smaller G) or one fewer (larger G) -- if
    // that keeps G within [3/4, 4/3] of the budget's G: much smaller groups put more
    // workgroups on each event's table slot and counter (8 MiB events at MTU 9000 lose
    // 9 % at G 16 -> 10). 205 x 1 MiB at MTU 1500: G 64 -> 49, 2342 -> 3059 groups,
    // reas_kernel 79.0 -> 77.6 us.
    {
        const uint32_t cap = NT == kReasNTSmall ? reas_resident_groups<U, kReasNTSmall>()
                           : NT == kReasNTJumbo ? reas_resident_groups<U, kReasNTJumbo>()
                                                : reas_resident_groups<U, kBlock>();
        if (cap) {
            const uint32_t G0 = G, waves = cdiv(cdiv(n, G0), cap);
            uint32_t best = G0, bestDev = ~0u;
            for (uint32_t k = (waves > 1 ? waves - 1 : waves); k <= waves; k++) {
                const uint32_t c = cdiv(n, k * cap);
                if (c > 64 || 4u * c < 3u * G0 || 3u * c > 4u * G0) continue;
                const uint32_t dev = c > G0 ? c - G0 : G0 - c;
                if (dev < bestDev) best = c, bestDev = dev;
            }
            G = best;
        }
    }
    return G;
}

// The jumbo-slot launch (512 threads) at most 2 workgroups per CU (16 waves instead of 24):
// MTU 9000 reas_kernel 71.2 -> 69.3 us (profiles/round4/ab/jumbo_cold_caps.log); the
// 768-thread launch is at 2 per CU by its registers already, and a cap there changes
// nothing (reas_caps.log).
constexpr uint32_t kReasJumboPerCU = 2;

hipError_t launch_reassemble(const ReasDev &R, const uint8_t *pkts, uint32_t stride,
                             const uint32_t *lens, uint32_t n, uint64_t now, hipStream_t stream)
{
    constexpr int U = kReasU;
    if (n == 0) return hipSuccess;
    const int NT = reas_threads(stride);
    const uint32_t G = reas_group_size(n, stride, R.groupSize, NT);
    const uint32_t groups = cdiv(n, G);
    if (stride <= 4096u)
        hipLaunchKernelGGL((reas_kernel<U, kReasNTSmall>), dim3(groups), dim3(kReasNTSmall), 0, stream, R,
                           pkts, stride, lens, n, now, G, (const uint32_t *)nullptr);
    else
        hipLaunchKernelGGL((reas_kernel<U, kReasNTJumbo>), dim3(groups), dim3(kReasNTJumbo),
                           occupancy_lds(reas_kernel<U, kReasNTJumbo>, kReasJumboPerCU), stream, R,
                           pkts, stride, lens, n, now, G, (const uint32_t *)nullptr);
    return hipGetLastError();
}

#if E2SAR_HIP_EXPERIMENTAL
hipError_t launch_reassemble_groups(const ReasDev &R, const uint8_t *pkts, uint32_t stride, const uint32_t *lens,
                                    uint32_t n, const uint32_t *starts, uint32_t nGroups, uint64_t now,
                                    hipStream_t stream)
{
    constexpr int U = kReasU;
    if (n == 0 || nGroups == 0) return hipSuccess;
    hipLaunchKernelGGL((reas_kernel<U, kBlock>), dim3(nGroups), dim3(kBlock), 0, stream, R, pkts, stride, lens, n, now, 64u,
                       starts);
    return hipGetLastError();
}

hipError_t launch_segreas(ChainBatches cb, int lbVersion, uint32_t maxPld, uint32_t stride, const ReasDev &R,
                          uint64_t now, hipStream_t stream)
{
    constexpr int U = kReasU;
    if (cb.nb == 0 || cb.nb > kChainMaxBatches) return hipErrorInvalidValue;
    uint64_t grid = 0;
    for (uint32_t b = 0; b < cb.nb; b++) {
        ChainBatch &B = cb.b[b];
        const uint64_t chunks = (uint64_t)B.maxPacketsPerEvent * (stride >> 4);
        if (chunks > 0xFFFFFFFFull) return hipErrorInvalidValue;
        B.bpe = (B.nEvents && B.n) ? cdiv(chunks, (uint64_t)kBlock * kChainSegU) : 0u;
        B.G = B.n ? reas_group_size(B.n, stride, R.groupSize, kBlock) : 1u;
        B.start = (uint32_t)grid;
        B.nSeg = B.bpe * B.nEvents;
        grid += (uint64_t)B.nSeg + (B.n ? cdiv(B.n, B.G) : 0u);
        if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
    }
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL((segreas_kernel<U>), dim3((uint32_t)grid), dim3(kBlock), 0, stream, cb, lbVersion, maxPld, stride,
                       R, now);
    return hipGetLastError();
}

#endif  // E2SAR_HIP_EXPERIMENTAL

hipError_t launch_reas_classify(const ReasDev &R, const uint8_t *pkts, uint32_t stride, const uint32_t *lens,
                                uint32_t n, uint64_t now, void *work, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    uint8_t *w = static_cast<uint8_t *>(work);
    hipLaunchKernelGGL(reas_classify_kernel, dim3(cdiv(n, kBlock)), dim3(kBlock), 0, stream, R, pkts, stride, lens,
                       n, now, reinterpret_cast<PktInfo *>(w), reinterpret_cast<FinishRec *>(w + work_fin_off(n)));
    return hipGetLastError();
}

// Staged stores (scatter_group<..., STAGE>: a one-round group's chunks pass through LDS so
// every event store is a whole aligned 16-byte store) per launch.  Measured per user,
// interleaved on one box (profiles/round4/ab/scatter_stores_*.log): config 3's split scatter
// (MTU 9000, streaming) 232.0-232.3 vs 235.9-236.4 us; cold leg at MTU 9000 83.4 vs 84.9-86.4
// us; hot split scatter at MTU 1500 67.3-67.5 vs 68.5-68.7 us; reference-order batches
// 123.0-123.6 vs 125.2-125.4 us; but the cold leg at MTU 1500 (8-datagram groups read from
// HBM, where the LDS barrier waits for the slowest of the group's loads) 84.9-85.5 vs
// 83.0-83.3 us.  So: staged unless the datagrams stream in at small strides.
static bool scatter_stage(uint32_t stride, bool nt) { return !nt || stride > 2048u; }

// An unstaged streaming scatter launch (cold datagrams at small strides) at most 6
// workgroups per CU instead of 8.  Round 4, cold leg at MTU 1500
// (profiles/round4/ab/scatter_occupancy.log): 82.7 vs 83.5-83.9 us per pipelined launch at
// 6 per CU, 84.8-86.0 at 5, 88.0-88.8 at 4; staged launches (their own 18 KiB of LDS) lose
// with any cap (config 3 284-286 vs 232 us at 3 per CU), so they keep none.
constexpr uint32_t kColdScatterPerCU = 6;
template <typename K>
static size_t scatter_lds(K kernel, bool stage, bool nt)
{
    return (!stage && nt) ? occupancy_lds(kernel, kColdScatterPerCU) : 0;
}

hipError_t launch_reas_scatter(const ReasDev &R, const uint8_t *pkts, uint32_t stride, uint32_t n,
                               const void *work, hipStream_t stream, bool nt)
{
    if (n == 0) return hipSuccess;
    const uint8_t *w = static_cast<const uint8_t *>(work);
    uint32_t blocks = 0;
    const uint32_t G = scatter_geometry(stride, n, blocks);
    const PktInfo *info = reinterpret_cast<const PktInfo *>(w);
    const FinishRec *fin = reinterpret_cast<const FinishRec *>(w + work_fin_off(n));
    const bool st = scatter_stage(stride, nt);
    auto go = [&](auto kernel) {
        hipLaunchKernelGGL(kernel, dim3(blocks), dim3(scatter_tb(stride)), scatter_lds(kernel, st, nt), stream, R, pkts, stride,
                           n, G, info, fin);
    };
    constexpr int U = kScatU, UJ = kScatUJumbo;
    constexpr int TJ = kScatBlockJumbo;
    if (scatter_u(stride) == UJ) nt ? go(reas_scatter_kernel<UJ, true, true, TJ>) : go(reas_scatter_kernel<UJ, false, true, TJ>);
    else if (nt) st ? go(reas_scatter_kernel<U, true, true>) : go(reas_scatter_kernel<U, true, false>);
    else st ? go(reas_scatter_kernel<U, false, true>) : go(reas_scatter_kernel<U, false, false>);
    return hipGetLastError();
}

hipError_t launch_reas_scatter_classify(const ReasDev &R, uint32_t stride, const uint8_t *spk, uint32_t sn,
                                        const void *swork, const uint8_t *cpk, const uint32_t *clens, uint32_t cn,
                                        uint64_t now, void *cwork, hipStream_t stream, bool nt)
{
    if (cn == 0) return launch_reas_scatter(R, spk, stride, sn, swork, stream, nt);
    if (sn == 0) return launch_reas_classify(R, cpk, stride, clens, cn, now, cwork, stream);
    const uint8_t *sw = static_cast<const uint8_t *>(swork);
    uint8_t *cw = static_cast<uint8_t *>(cwork);
    uint32_t sblocks = 0;
    const uint32_t G = scatter_geometry(stride, sn, sblocks);
    const uint32_t nCls = (cdiv(cn, (uint32_t)scatter_tb(stride)) + 7u) & ~7u;     // multiples of 8: see xcd_runs
    // where the classify workgroups sit in the grid: kPipeClsAtPercent of the way
    // through the scatter workgroups.  At the front (0, round 2's form) they hold ~590
    // workgroup slots through their dependent round trips while the scatter ramps up; three
    // quarters of the way in they run beside the scatter's last quarter and finish with it
    // (cold leg, 205 x 1 MiB: 81.4-83.8 vs 83.9-87.0 us per launch over three boxes, 50 / 65 /
    // 80 / 88 % in between; profiles/round3/s3_cls/)
    const uint32_t clsStart = (uint32_t)((uint64_t)sblocks * kPipeClsAtPercent / 100u) & ~7u;
    const bool st = scatter_stage(stride, nt);
    auto go = [&](auto kernel) {
        hipLaunchKernelGGL(kernel, dim3(nCls + sblocks), dim3(scatter_tb(stride)), scatter_lds(kernel, st, nt), stream, R, stride,
                           spk, sn, G,
                           reinterpret_cast<const PktInfo *>(sw),
                           reinterpret_cast<const FinishRec *>(sw + work_fin_off(sn)), cpk, clens, cn, now,
                           reinterpret_cast<PktInfo *>(cw), reinterpret_cast<FinishRec *>(cw + work_fin_off(cn)), nCls,
                           clsStart);
    };
    constexpr int U = kScatU, UJ = kScatUJumbo;
    constexpr int TJ = kScatBlockJumbo;
    if (scatter_u(stride) == UJ)
        nt ? go(reas_scatter_classify_kernel<UJ, true, true, TJ>) : go(reas_scatter_classify_kernel<UJ, false, true, TJ>);
    else if (nt) st ? go(reas_scatter_classify_kernel<U, true, true>) : go(reas_scatter_classify_kernel<U, true, false>);
    else st ? go(reas_scatter_classify_kernel<U, false, true>) : go(reas_scatter_classify_kernel<U, false, false>);
    return hipGetLastError();
}

hipError_t launch_ro_classify(const ReasDev &R, const uint8_t *pkts, uint32_t stride, const uint32_t *lens,
                              uint32_t n, uint64_t now, void *work, void *scratch, size_t scratchBytes,
                              hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    if (ro_scratch_bytes(n, R.tableSlots) > scratchBytes) return hipErrorInvalidValue;
    uint8_t *w = static_cast<uint8_t *>(work);
    PktInfo *info = reinterpret_cast<PktInfo *>(w);
    const RoScratch sc = ro_scratch_layout(scratch, n, R.tableSlots);
    hipLaunchKernelGGL((ro_key_kernel<kRoKeyBlock>), dim3(cdiv(n, (uint32_t)kRoKeyBlock)), dim3(kRoKeyBlock), 0, stream,
                       R, pkts, stride, lens, n, now, sc, info);
    hipLaunchKernelGGL(ro_place_kernel, dim3(kPlaceBlocks), dim3(kPlaceThreads), 0, stream, sc, R.tableSlots, n);
    // one wave per key: at most min(n, tableSlots) keys
    const uint32_t waves = n < R.tableSlots ? n : R.tableSlots;
    hipLaunchKernelGGL((ro_walk_kernel<1, kRoWalkLds>), dim3(waves), dim3(64), 0, stream, R, sc, R.tableSlots, now, info,
                       reinterpret_cast<FinishRec *>(w + work_fin_off(n)));
    return hipGetLastError();
}

hipError_t launch_gc(const ReasDev &R, uint64_t now, uint64_t timeout, hipStream_t stream)
{
    hipLaunchKernelGGL(reas_gc_kernel, dim3(cdiv(R.tableSlots, kBlock)), dim3(kBlock), 0, stream, R,
                       now, timeout);
    return hipGetLastError();
}

hipError_t launch_recycle(const ReasDev &R, bool dropCompleted, hipStream_t stream)
{
    hipLaunchKernelGGL(reas_recycle_kernel, dim3(cdiv(R.tableSlots, kBlock)), dim3(kBlock), 0, stream,
                       R, dropCompleted ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_compact(const ReasDev &from, const ReasDev &to, hipStream_t stream)
{
    hipError_t e = launch_zero_words(to.slots, sizeof(ReasSlot) / 4 * (uint64_t)to.tableSlots, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(reas_compact_kernel, dim3(from.tableSlots), dim3(kBlock), 0, stream, from, to);
    hipLaunchKernelGGL(reas_compact_finish, dim3(1), dim3(1), 0, stream, to);
    return hipGetLastError();
}


// ---------------------------------------------------------------------------------
// multi-GPU: route a landed datagram batch to the rank that owns each event
//
// owner(eventNum) = eventNum % world.  Datagrams that cannot be parsed stay
// on this rank (so their badHeaderDiscards are counted where they landed).  The packing
// is stable: datagrams keep their landing order inside each destination's span, so an
// in-order stream stays in order after the exchange.

constexpr uint32_t kMaxWorld = 64;

__device__ __forceinline__ uint32_t route_dest(const uint8_t *pkts, uint32_t stride, const uint32_t *lens,
                                               uint32_t p, int withLB, uint32_t world, uint32_t self)
{
    const uint32_t hl = withLB ? kLBREHdrLen : kREHdrLen;
    const uint32_t len = lens[p];
    if (len < hl || len > stride) return self;
    const uint8_t *re = pkts + (uint64_t)p * stride + (withLB ? kLBHdrLen : 0u);
    const u32x4 w = ld16(re);
    if (!re_valid(w.x)) return self;
    const uint64_t ev = ((uint64_t)bswap32(w.w) << 32) | bswap32(ld4(re + 16));
    return (uint32_t)(ev % world);
}

constexpr uint32_t kNoDest = 0xFFFFFFFFu;

// Destination of datagram p, or kNoDest past the batch and -- foreign-only routing
// (excludeSelf) -- for every datagram that stays here (owned here, or unparsable): those
// are reassembled where they landed by a reassembler set to this rank's ownership.
__device__ __forceinline__ uint32_t route_dest_x(const uint8_t *pkts, uint32_t stride, const uint32_t *lens,
                                                 uint32_t p, uint32_t n, int withLB, uint32_t world, uint32_t self,
                                                 int excludeSelf)
{
    if (p >= n) return kNoDest;
    const uint32_t d = route_dest(pkts, stride, lens, p, withLB, world, self);
    return (excludeSelf && d == self) ? kNoDest : d;
}

// per-block, per-destination counts (wave ballots, deterministic)
__global__ __launch_bounds__(kBlock) void route_hist_kernel(const uint8_t *__restrict__ pkts, uint32_t stride,
                                                            const uint32_t *__restrict__ lens, uint32_t n, int withLB,
                                                            uint32_t world, uint32_t self, int excludeSelf,
                                                            uint32_t *__restrict__ blockHist)
{
    __shared__ uint32_t cnt[kMaxWorld];
    for (uint32_t d = threadIdx.x; d < world; d += kBlock) cnt[d] = 0;
    __syncthreads();
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t dest = route_dest_x(pkts, stride, lens, p, n, withLB, world, self, excludeSelf);
    for (uint32_t d = 0; d < world; d++) {
        const uint64_t m = __ballot(dest == d);
        if ((threadIdx.x & 63) == 0 && m) atomicAdd(&cnt[d], (uint32_t)__builtin_popcountll(m));
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < world; d += kBlock) blockHist[(uint64_t)blockIdx.x * world + d] = cnt[d];
}

// one block: exclusive scans -> per-block bases, per-destination counts and bases.
// For each destination the nBlocks counts are scanned 256 at a time (wave prefix sums
// through LDS, a running carry between tiles), so the scan costs nBlocks/256 block steps
// per destination instead of nBlocks dependent loads.
// Append mode (cap > 0): rank d's span is a region of cap slots at d * cap that successive
// batches append to; destBase[d] = d * cap + running[d], then running[d] += this batch's
// count (the count keeps growing past cap, so the caller sees an overflow; the pack kernel
// writes nothing past a region's end).  counts may be NULL in append mode.
__global__ __launch_bounds__(kBlock) void route_scan_kernel(uint32_t *__restrict__ blockHist, uint32_t nBlocks,
                                                            uint32_t world, uint32_t *__restrict__ counts,
                                                            uint32_t *__restrict__ destBase, uint32_t cap,
                                                            uint32_t *__restrict__ running)
{
    __shared__ uint32_t waveSum[kBlock / 64];
    __shared__ uint32_t tot[kMaxWorld];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    for (uint32_t d = 0; d < world; d++) {
        uint32_t carry = 0;
        for (uint32_t b0 = 0; b0 < nBlocks; b0 += kBlock) {
            const uint32_t b = b0 + threadIdx.x;
            const uint32_t c = (b < nBlocks) ? blockHist[(uint64_t)b * world + d] : 0u;
            uint32_t inc = c;                                 // inclusive scan in the wave
#pragma unroll
            for (uint32_t o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, o);
                if (lane >= o) inc += y;
            }
            if (lane == 63) waveSum[wv] = inc;
            __syncthreads();
            uint32_t before = carry;
            for (uint32_t w = 0; w < wv; w++) before += waveSum[w];
            if (b < nBlocks) blockHist[(uint64_t)b * world + d] = before + inc - c;
            uint32_t tile = 0;
            for (uint32_t w = 0; w < kBlock / 64; w++) tile += waveSum[w];
            carry += tile;
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            tot[d] = carry;
            if (counts) counts[d] = carry;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t d = 0; d < world; d++) {
            if (cap) {
                const uint32_t have = running[d];
                destBase[d] = d * cap + have;
                running[d] = have + tot[d];
            } else {
                destBase[d] = run;
                run += tot[d];
            }
        }
    }
}

// copy every datagram slot (stride bytes) to its place in the send buffer.  Workgroup
// (g, s) = blockIdx (g * kPackSplit + s) recomputes the places of datagrams [256g, 256g+256)
// (header reads that hit in L2) and copies the s-th of kPackSplit slices of their chunks.
// A/B at 205 x 1 MiB, MTU 1500, spread landing (route = hist + scan + pack, per batch):
// split 1/2/4/8 -> 97/92/100/116 us with non-temporal datagram loads, which also leave the
// Infinity Cache to the packed copy that reassembly reads next (reas 108 -> 79 us).
constexpr uint32_t kPackSplit = 2;
__global__ __launch_bounds__(kBlock) void route_pack_kernel(const uint8_t *__restrict__ pkts, uint32_t stride,
                                                            const uint32_t *__restrict__ lens, uint32_t n, int withLB,
                                                            uint32_t world, uint32_t self, int excludeSelf,
                                                            const uint32_t *__restrict__ blockBase,
                                                            const uint32_t *__restrict__ destBase, uint32_t cap,
                                                            uint8_t *__restrict__ out, uint32_t *__restrict__ outLens)
{
    __shared__ uint32_t pos[kBlock];
    __shared__ uint32_t waveCnt[kBlock / 64][kMaxWorld];
    const uint32_t g = blockIdx.x / kPackSplit, sl = blockIdx.x % kPackSplit;
    const uint32_t p = g * kBlock + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t dest = route_dest_x(pkts, stride, lens, p, n, withLB, world, self, excludeSelf);
    uint32_t rank = 0;
    for (uint32_t d = 0; d < world; d++) {
        const uint64_t m = __ballot(dest == d);
        if (dest == d) rank = (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
        if (lane == 0) waveCnt[wv][d] = (uint32_t)__builtin_popcountll(m);
    }
    __syncthreads();
    pos[threadIdx.x] = kNoDest;
    if (dest != kNoDest) {
        uint32_t before = 0;
        for (uint32_t w = 0; w < wv; w++) before += waveCnt[w][dest];
        const uint32_t q = destBase[dest] + blockBase[(uint64_t)g * world + dest] + before + rank;
        if (!cap || q < (dest + 1u) * cap) {                  // append mode: nothing past the region
            pos[threadIdx.x] = q;
            if (sl == 0) outLens[q] = lens[p];
        }
    }
    // foreign-only routing leaves most blocks with nothing to move at small world sizes
    if (!__syncthreads_or(dest != kNoDest)) return;
    const uint32_t p0 = g * kBlock;
    const uint32_t np = (n - p0 < kBlock) ? n - p0 : kBlock;
    const uint32_t spc = stride >> 4;
    const uint32_t nch = np * spc;
    const float rspc = 1.0f / (float)spc;
    // this workgroup's slice of the chunks, in two-phase rounds of 4 chunks per thread
    const uint32_t c0 = (uint32_t)((uint64_t)nch * sl / kPackSplit);
    const uint32_t c1 = (uint32_t)((uint64_t)nch * (sl + 1) / kPackSplit);
    constexpr int UR = 4;
    for (uint32_t r0 = c0; r0 < c1; r0 += kBlock * UR) {
        u32x4 x[UR];
        uint32_t qq[UR], cc[UR];
#pragma unroll
        for (int u = 0; u < UR; u++) {
            const uint32_t i = r0 + (uint32_t)u * kBlock + threadIdx.x;
            const uint32_t ic = (i < c1) ? i : c0;
            uint32_t k = (uint32_t)((float)ic * rspc);
            if (k * spc > ic) k--;
            else if ((k + 1u) * spc <= ic) k++;
            cc[u] = ic - k * spc;
            qq[u] = (i < c1) ? pos[k] : kNoDest;                       // kNoDest: stays here
            x[u] = u32x4{0u, 0u, 0u, 0u};
            if (qq[u] != kNoDest)
                x[u] = ld16_nt(pkts + (uint64_t)(p0 + k) * stride + 16u * cc[u]);
        }
#pragma unroll
        for (int u = 0; u < UR; u++) {
            if (qq[u] != kNoDest) {
                uint8_t *o = out + (uint64_t)qq[u] * stride + 16u * cc[u];
                st16(o, x[u]);
            }
        }
    }
}

// Append routing in ONE launch (e2sar_hip_route_append): a workgroup of 256 datagrams counts
// its datagrams per destination (wave ballots), reserves room in each destination's region
// with one atomicAdd on that region's counter, and copies its datagrams there -- no
// histogram / scan launches in front of the copy (three dependent launches cost ~20 us per
// batch even when nothing is foreign).  Within a workgroup a destination's datagrams keep
// their order; workgroups append in the order they reserve.
__global__ __launch_bounds__(kBlock) void route_append_kernel(const uint8_t *__restrict__ pkts, uint32_t stride,
                                                              const uint32_t *__restrict__ lens, uint32_t n, int withLB,
                                                              uint32_t world, uint32_t self, int excludeSelf, uint32_t cap,
                                                              uint32_t *__restrict__ running, uint8_t *__restrict__ out,
                                                              uint32_t *__restrict__ outLens)
{
    __shared__ uint32_t pos[kBlock];
    __shared__ uint32_t waveCnt[kBlock / 64][kMaxWorld];
    __shared__ uint32_t base[kMaxWorld];
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t dest = route_dest_x(pkts, stride, lens, p, n, withLB, world, self, excludeSelf);
    uint32_t rank = 0;
    for (uint32_t d = 0; d < world; d++) {
        const uint64_t m = __ballot(dest == d);
        if (dest == d) rank = (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
        if (lane == 0) waveCnt[wv][d] = (uint32_t)__builtin_popcountll(m);
    }
    __syncthreads();
    if (threadIdx.x < world) {
        uint32_t tot = 0;
        for (uint32_t w = 0; w < kBlock / 64; w++) tot += waveCnt[w][threadIdx.x];
        base[threadIdx.x] = tot ? atomicAdd(&running[threadIdx.x], tot) : 0u;
    }
    __syncthreads();
    uint32_t q = kNoDest;
    if (dest != kNoDest) {
        uint32_t before = 0;
        for (uint32_t w = 0; w < wv; w++) before += waveCnt[w][dest];
        const uint32_t r = base[dest] + before + rank;
        if (r < cap) {                                        // nothing past the region; running still counts it
            q = dest * cap + r;
            outLens[q] = lens[p];
        }
    }
    pos[threadIdx.x] = q;
    if (!__syncthreads_or(q != kNoDest)) return;
    const uint32_t p0 = blockIdx.x * kBlock;
    const uint32_t np = (n - p0 < kBlock) ? n - p0 : kBlock;
    const uint32_t spc = stride >> 4;
    const uint32_t nch = np * spc;
    const float rspc = 1.0f / (float)spc;
    constexpr int UR = 4;
    for (uint32_t r0 = 0; r0 < nch; r0 += kBlock * UR) {
        u32x4 x[UR];
        uint32_t qq[UR], cc[UR];
#pragma unroll
        for (int u = 0; u < UR; u++) {
            const uint32_t i = r0 + (uint32_t)u * kBlock + threadIdx.x;
            const uint32_t ic = (i < nch) ? i : 0u;
            uint32_t k = (uint32_t)((float)ic * rspc);
            if (k * spc > ic) k--;
            else if ((k + 1u) * spc <= ic) k++;
            cc[u] = ic - k * spc;
            qq[u] = (i < nch) ? pos[k] : kNoDest;
            x[u] = u32x4{0u, 0u, 0u, 0u};
            if (qq[u] != kNoDest)
                x[u] = ld16_nt(pkts + (uint64_t)(p0 + k) * stride + 16u * cc[u]);
        }
#pragma unroll
        for (int u = 0; u < UR; u++) {
            if (qq[u] != kNoDest) {
                uint8_t *o = out + (uint64_t)qq[u] * stride + 16u * cc[u];
                st16(o, x[u]);
            }
        }
    }
}

hipError_t launch_route_append(const uint8_t *pkts, uint32_t stride, const uint32_t *lens, uint32_t n, int withLB,
                               uint32_t world, uint32_t self, int excludeSelf, uint8_t *out, uint32_t *outLens,
                               uint32_t cap, uint32_t *running, hipStream_t stream)
{
    if (world == 0 || world > kMaxWorld || self >= world || cap == 0) return hipErrorInvalidValue;
    if ((uint64_t)cap * world > 0xFFFFFFFFull) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(route_append_kernel, dim3(cdiv(n, kBlock)), dim3(kBlock), 0, stream, pkts, stride, lens, n, withLB,
                       world, self, excludeSelf, cap, running, out, outLens);
    return hipGetLastError();
}

size_t route_workspace_bytes(uint32_t n, uint32_t world)
{
    const uint64_t nb = (n + kBlock - 1) / kBlock;
    return (size_t)((nb * world + world) * sizeof(uint32_t));
}

hipError_t launch_route(const uint8_t *pkts, uint32_t stride, const uint32_t *lens, uint32_t n, int withLB,
                        uint32_t world, uint32_t self, int excludeSelf, uint8_t *out, uint32_t *outLens,
                        uint32_t *counts, void *workspace, hipStream_t stream, uint32_t cap, uint32_t *running)
{
    if (world == 0 || world > kMaxWorld || self >= world) return hipErrorInvalidValue;
    if (cap && (uint64_t)cap * world > 0xFFFFFFFFull) return hipErrorInvalidValue;
    if (n == 0) return counts ? launch_zero_words(counts, world, stream) : hipSuccess;
    const uint32_t nb = cdiv(n, kBlock);
    uint32_t *blockHist = static_cast<uint32_t *>(workspace);
    uint32_t *destBase = blockHist + (size_t)nb * world;
    hipLaunchKernelGGL(route_hist_kernel, dim3(nb), dim3(kBlock), 0, stream, pkts, stride, lens, n, withLB, world,
                       self, excludeSelf, blockHist);
    hipLaunchKernelGGL(route_scan_kernel, dim3(1), dim3(kBlock), 0, stream, blockHist, nb, world, counts, destBase,
                       cap, running);
    hipLaunchKernelGGL(route_pack_kernel, dim3(nb * kPackSplit), dim3(kBlock), 0, stream, pkts, stride, lens, n, withLB, world,
                       self, excludeSelf, blockHist, destBase, cap, out, outLens);
    return hipGetLastError();
}

}  // namespace e2sar_amd

#if E2SAR_TRACE
// Experiment builds only: copy the timeline of the last reas_kernel (k = 0) or seg_kernel
// (k = 1) launch, 4 words per workgroup, to host memory.
extern "C" int e2sar_hip_debug_trace(int k, uint64_t *out, size_t words)
{
    if (k < 0 || k > 2 || words > e2sar_amd::kTraceBlocks * 4) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(e2sar_amd::g_trace), words * 8, (size_t)k * e2sar_amd::kTraceBlocks * 4 * 8,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int e2sar_hip_debug_trace_clear(void)
{
    static uint64_t zero[3 * e2sar_amd::kTraceBlocks * 4];
    return hipMemcpyToSymbol(HIP_SYMBOL(e2sar_amd::g_trace), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
