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

namespace e2sar_amd {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(4))) u32x4_a4;   // 16-byte access at dword alignment

constexpr int kBlock = 256;

// Global-address-space accessors: the event/packet/arena pointers reach the kernels
// through descriptor tables, so without these hipcc falls back to flat_* accesses.
#define E2SAR_GLOBAL __attribute__((address_space(1)))
__device__ __forceinline__ u32x4 ld16(const uint8_t *p) { return *(const E2SAR_GLOBAL u32x4_a4 *)(p); }
__device__ __forceinline__ void st16(uint8_t *p, u32x4 v) { *(E2SAR_GLOBAL u32x4 *)(p) = v; }
__device__ __forceinline__ uint32_t ld4(const uint8_t *p) { return *(const E2SAR_GLOBAL uint32_t *)(p); }
__device__ __forceinline__ void st4(uint8_t *p, uint32_t v) { *(E2SAR_GLOBAL uint32_t *)(p) = v; }
__device__ __forceinline__ uint8_t ld1(const uint8_t *p) { return *(const E2SAR_GLOBAL uint8_t *)(p); }
__device__ __forceinline__ void st1(uint8_t *p, uint8_t v) { *(E2SAR_GLOBAL uint8_t *)(p) = v; }

// ---------------------------------------------------------------------------------
// segmentation

__device__ __forceinline__ uint32_t hdr_word(const HdrWords &h, uint32_t idx)
{
    // idx in [0, 9); small select chain (runs only on header/edge chunks)
    uint32_t r = h.w[0];
#pragma unroll
    for (uint32_t i = 1; i < 9; i++) r = (idx == i) ? h.w[i] : r;
    return r;
}

__device__ __forceinline__ uint32_t low_bytes_mask(uint32_t n)   // n in [1,3]
{
    return (n >= 4) ? 0xFFFFFFFFu : ((1u << (8 * n)) - 1u);
}

// One 16-byte chunk c of datagram k of an event; `pl` = first payload byte of the
// datagram, L = its payload length.  Returns false when the chunk lies wholly past the
// datagram end (nothing to store).
template <bool A4>
__device__ __forceinline__ bool seg_chunk(u32x4 &v, const HdrWords &h, const uint8_t *pl,
                                          uint32_t L, uint32_t c)
{
    const uint32_t q0 = 16u * c;
    const uint32_t dlen = kLBREHdrLen + L;
    if (q0 >= dlen) return false;
    if (A4 && c >= 3 && q0 + 16u <= dlen) {
        v = ld16(pl + (q0 - kLBREHdrLen));
        return true;
    }
    if (A4) {
#pragma unroll
        for (uint32_t d = 0; d < 4; d++) {
            const uint32_t q = q0 + 4u * d;
            uint32_t w;
            if (q < kLBREHdrLen) {
                w = hdr_word(h, q >> 2);
            } else {
                const uint32_t r = q - kLBREHdrLen;
                if (r >= L) {
                    w = 0;
                } else {
                    w = ld4(pl + r);
                    if (r + 4u > L) w &= low_bytes_mask(L - r);
                }
            }
            v[d] = w;
        }
    } else {
        // generic byte path: any event alignment, any maxPldLen
#pragma unroll
        for (uint32_t d = 0; d < 4; d++) {
            uint32_t w = 0;
#pragma unroll
            for (uint32_t b = 0; b < 4; b++) {
                const uint32_t q = q0 + 4u * d + b;
                uint32_t byte;
                if (q < kLBREHdrLen) byte = (hdr_word(h, q >> 2) >> (8 * (q & 3))) & 0xFFu;
                else if (q - kLBREHdrLen < L) byte = ld1(pl + (q - kLBREHdrLen));
                else byte = 0;
                w |= byte << (8 * b);
            }
            v[d] = w;
        }
    }
    return true;
}

// grid.x = nEvents * blocksPerEvent; each block owns kBlock*U consecutive 16-byte
// chunks of ONE event's datagram range (event-major: every event field is a scalar).
template <bool A4, int U>
__global__ __launch_bounds__(kBlock) void seg_kernel(const e2sar_hip_seg_event *__restrict__ events,
                                                     uint32_t blocksPerEvent, int lbVersion,
                                                     uint32_t maxPld, uint8_t *__restrict__ pkts,
                                                     uint32_t stride, uint32_t *__restrict__ lens)
{
    const uint32_t e = blockIdx.x / blocksPerEvent;
    const uint32_t bx = blockIdx.x - e * blocksPerEvent;
    const e2sar_hip_seg_event ev = events[e];
    const uint32_t bytes = ev.bytes;
    const uint32_t npk = (bytes + maxPld - 1u) / maxPld;
    const uint32_t spc = stride >> 4;
    const uint32_t nch = npk * spc;
    const uint32_t j0 = bx * (uint32_t)(kBlock * U);
    if (j0 >= nch) return;

    u32x4 v[U];
    uint8_t *dst[U];
    bool st[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t j = j0 + (uint32_t)u * kBlock + threadIdx.x;
        st[u] = false;
        dst[u] = nullptr;
        if (j < nch) {
            const uint32_t k = j / spc;
            const uint32_t c = j - k * spc;
            const uint64_t off = (uint64_t)k * maxPld;
            const uint32_t L = (bytes - off > maxPld) ? maxPld : (uint32_t)(bytes - off);
            HdrWords h;
            lbre_words(h, lbVersion, ev.entropy, ev.lbTick, ev.dataId, (uint32_t)off, bytes,
                       ev.eventNum);
            const uint64_t p = (uint64_t)ev.pktBase + k;
            dst[u] = pkts + p * stride + 16u * c;
            st[u] = seg_chunk<A4>(v[u], h, ev.data + off, L, c);
            if (c == 0 && lens) lens[p] = kLBREHdrLen + L;
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++)
        if (st[u]) st16(dst[u], v[u]);
}

// ---------------------------------------------------------------------------------
// reassembly: event table protocol
//
// slot.state: EMPTY -> BUSY (CAS by the inserting lane) -> READY (after the key,
// length and buffer offset are stored) -> DONE (completed) / LOST (GC'd).  Every
// cross-lane hand-off of slot fields uses agent-scope atomic loads/stores (sc1) with
// the publishing lane's own s_waitcnt vmcnt(0) before the READY store
// (MI355X_MICROARCH.md 'Valid forms', R1 row: one storing lane, sc1 payload + flag).

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

__device__ LookupResult find_or_create(const ReasDev &R, uint64_t ev, uint32_t d,
                                       uint32_t blen, uint64_t now)
{
    LookupResult res{kNoSlot, 0, kNoBuf};
    const uint32_t mask = R.tableSlots - 1u;
    uint32_t h = slot_hash(ev, d, mask);
    for (uint32_t probe = 0; probe < R.tableSlots; probe++, h = (h + 1u) & mask) {
        ReasSlot *sl = R.slots + h;
        uint32_t stt = ld_agent(&sl->state);
        if (stt == kEmpty) {
            const uint32_t old = atomicCAS(&sl->state, (uint32_t)kEmpty, (uint32_t)kBusy);
            if (old == kEmpty) {
                // this lane owns the slot: publish key, length, buffer, then READY
                const uint64_t need = ((uint64_t)blen + 255ull) & ~255ull;
                uint64_t boff = atomicAdd(&R.ctl->arenaTop, (unsigned long long)(need ? need : 256ull));
                if (boff + blen > R.arenaBytes) {
                    boff = kNoBuf;
                    atomicOr(&R.ctl->errorFlags, 2u);
                }
                st_agent(&sl->eventNum, ev);
                st_agent(&sl->dataId, d);
                st_agent(&sl->bytes, blen);
                st_agent(&sl->bufOff, boff);
                st_agent(&sl->created, now);
                st_agent(&sl->acc, 0ull);
                atomicAdd(reinterpret_cast<unsigned long long *>(&R.ctl->inProgress), 1ull);
                atomicAdd(&R.ctl->tableUsed, 1u);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                st_agent(&sl->state, (uint32_t)kReady);
                res.slot = h;
                res.bytes = blen;
                res.bufOff = boff;
                return res;
            }
            stt = old;
        }
        uint32_t spins = 0;
        while (stt == kBusy) {
            __builtin_amdgcn_s_sleep(1);
            stt = ld_agent(&sl->state);
            if (++spins > kSpinLimit) {
                atomicOr(&R.ctl->errorFlags, 4u);
                return res;
            }
        }
        if (stt == kReady) {
            const uint64_t sev = ld_agent(&sl->eventNum);
            const uint32_t sd = ld_agent(&sl->dataId);
            if (sev == ev && sd == d) {
                res.slot = h;
                res.bytes = ld_agent(&sl->bytes);
                res.bufOff = ld_agent(&sl->bufOff);
                return res;
            }
        }
    }
    atomicOr(&R.ctl->errorFlags, 1u);
    return res;
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src)
{
    const uint32_t lo = __shfl((uint32_t)v, src);
    const uint32_t hi = __shfl((uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v, unsigned d)
{
    const uint32_t lo = __shfl_up((uint32_t)v, d);
    const uint32_t hi = __shfl_up((uint32_t)(v >> 32), d);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_down_u64(uint64_t v, unsigned d)
{
    const uint32_t lo = __shfl_down((uint32_t)v, d);
    const uint32_t hi = __shfl_down((uint32_t)(v >> 32), d);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += shfl_down_u64(v, o);
    return v;   // valid in lane 0
}

// One lane per datagram.  Consecutive lanes that carry the same (eventNum, dataId) form
// a run: only the run head touches the event table and only the run tail adds to the
// event's byte/fragment counter, so the per-event atomics are per run, not per packet.
__global__ __launch_bounds__(kBlock) void reas_classify(ReasDev R, const uint8_t *__restrict__ pkts,
                                                        uint32_t stride, const uint32_t *__restrict__ lens,
                                                        uint32_t n, uint64_t now,
                                                        PktInfo *__restrict__ info)
{
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool live = p < n;
    const uint32_t hl = R.withLB ? kLBREHdrLen : kREHdrLen;
    const uint32_t reo = R.withLB ? kLBHdrLen : 0u;

    uint32_t len = 0;
    bool ok = false, bad = false, derr = false;
    uint64_t ev = 0;
    uint32_t d = 0, off = 0, blen = 0, pl = 0;
    if (live) {
        len = lens[p];
        if (len < hl) {
            bad = true;                                       // too short to hold the headers
        } else if (len > stride) {
            derr = true;                                      // datagram overruns its slot
        } else {
            const uint32_t *re = reinterpret_cast<const uint32_t *>(pkts + (uint64_t)p * stride + reo);
            const uint32_t w0 = re[0], w1 = re[1], w2 = re[2], w3 = re[3], w4 = re[4];
            if (!re_valid(w0)) {
                bad = true;                                   // cpp:351-357
            } else {
                d = bswap16(w0 >> 16);
                off = bswap32(w1);
                blen = bswap32(w2);
                ev = ((uint64_t)bswap32(w3) << 32) | bswap32(w4);
                pl = len - hl;
                ok = true;
            }
        }
    }

    // ---- runs of equal keys ----
    const uint64_t pev = shfl_up_u64(ev, 1), nev = shfl_down_u64(ev, 1);
    const uint32_t pd = __shfl_up(d, 1), nd = __shfl_down(d, 1);
    const int pok = __shfl_up((int)ok, 1), nok = __shfl_down((int)ok, 1);
    const bool head = ok && (lane == 0 || !pok || pev != ev || pd != d);
    const bool tail = ok && (lane == 63 || !nok || nev != ev || nd != d);

    LookupResult lr{kNoSlot, 0, kNoBuf};
    if (head) lr = find_or_create(R, ev, d, blen, now);

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
    uint32_t xb = take ? pl : 0u, xc = take ? 1u : 0u;
    uint32_t ib = xb, ic = xc;
#pragma unroll
    for (unsigned s = 1; s < 64; s <<= 1) {
        const uint32_t yb = __shfl_up(ib, s), yc = __shfl_up(ic, s);
        if ((unsigned)lane >= s) {
            ib += yb;
            ic += yc;
        }
    }
    const uint32_t hb = __shfl(ib - xb, myhead), hc = __shfl(ic - xc, myhead);
    if (tail && slot != kNoSlot) {
        const uint32_t rb = ib - hb, rc = ic - hc;
        ReasSlot *sl = R.slots + slot;
        const uint64_t add = ((uint64_t)rc << kAccFragShift) | rb;
        const uint64_t old = atomicAdd(&sl->acc, (unsigned long long)add);
        const uint64_t nb = (old & kAccBytesMask) + rb;
        if (rc > 0 && nb == sbytes) {                          // curBytes == bytes (cpp:403)
            st_agent(&sl->state, (uint32_t)kDone);             // erase from the map (cpp:409)
            atomicAdd(&R.ctl->eventSuccess, 1ull);             // cpp:426
            atomicAdd(reinterpret_cast<unsigned long long *>(&R.ctl->inProgress), ~0ull);
            const uint32_t frags = (uint32_t)(old >> kAccFragShift) + rc;
            bool lostOnEnqueue = (boff == kNoBuf);
            if (!lostOnEnqueue) {
                const uint32_t idx = atomicAdd(&R.ctl->nCompleted, 1u);
                if (idx < R.queueCapacity) {
                    e2sar_hip_event_rec rec;
                    rec.eventNum = ev;
                    rec.arenaOffset = boff;
                    rec.bytes = sbytes;
                    rec.dataId = (uint16_t)d;
                    rec.flags = 0;
                    rec.numFragments = frags;
                    rec.reserved = 0;
                    R.completed[idx] = rec;
                } else {
                    lostOnEnqueue = true;                      // queue full (hpp:140-145)
                }
            }
            if (lostOnEnqueue) {
                atomicAdd(&R.ctl->enqueueLoss, 1ull);
                const uint32_t li = atomicAdd(&R.ctl->nLost, 1u);
                if (li < R.lostCapacity) {
                    e2sar_hip_lost_rec lr2;
                    lr2.eventNum = ev;
                    lr2.numFragments = frags;
                    lr2.dataId = (uint16_t)d;
                    lr2.enqueueLoss = 1;
                    lr2.reserved = 0;
                    R.lost[li] = lr2;
                }
            }
        }
    }

    if (live) {
        PktInfo pi;
        const bool scatter = take && boff != kNoBuf;
        pi.dst = scatter ? (uint64_t)(R.arena + boff + off) : 0ull;
        pi.plen = scatter ? pl : 0u;
        pi.hl = hl;
        info[p] = pi;
    }
    if (ok && slot == kNoSlot) derr = true;                    // table full / probe timeout

    // ---- stats: one atomic per wave per counter ----
    const uint64_t np = __builtin_popcountll(__ballot(live));
    const uint64_t nbad = __builtin_popcountll(__ballot(bad));
    const uint64_t nder = __builtin_popcountll(__ballot(derr));
    const uint64_t tb = wave_sum_u64(live ? (uint64_t)len : 0ull);
    if (lane == 0) {
        if (np) atomicAdd(&R.ctl->totalPackets, (unsigned long long)np);
        if (tb) atomicAdd(&R.ctl->totalBytes, (unsigned long long)tb);
        if (nbad) atomicAdd(&R.ctl->badHeaderDiscards, (unsigned long long)nbad);
        if (nder) atomicAdd(&R.ctl->dataErrCnt, (unsigned long long)nder);
    }
}

// ---------------------------------------------------------------------------------
// reassembly: payload scatter

__device__ __forceinline__ void copy_edge(uint8_t *lo, uint8_t *hi, const uint8_t *src)
{
    // [lo, hi) inside one 16-byte destination chunk; src corresponds to lo.
    const bool congruent = (((uintptr_t)lo ^ (uintptr_t)src) & 3u) == 0;
    while (lo < hi) {
        if (congruent && (((uintptr_t)lo & 3u) == 0) && lo + 4 <= hi) {
            st4(lo, ld4(src));
            lo += 4;
            src += 4;
        } else {
            st1(lo++, ld1(src++));
        }
    }
}

// Flat over the packet arena's 16-byte chunks: chunk c of packet p writes destination
// chunk (dst0 & ~15) + 16c, i.e. destination-aligned 16-byte stores.
template <int U>
__global__ __launch_bounds__(kBlock) void reas_scatter(const PktInfo *__restrict__ info,
                                                       const uint8_t *__restrict__ pkts,
                                                       uint32_t stride, uint32_t spc,
                                                       uint32_t nChunks)
{
    const uint32_t base = blockIdx.x * (uint32_t)(kBlock * U) + threadIdx.x;
    u32x4 v[U];
    uint8_t *dst[U];
    bool st[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t i = base + (uint32_t)u * kBlock;
        st[u] = false;
        dst[u] = nullptr;
        if (i < nChunks) {
            const uint32_t p = i / spc;
            const uint32_t c = i - p * spc;
            const PktInfo pi = info[p];
            if (pi.plen) {
                uint8_t *d0 = reinterpret_cast<uint8_t *>(pi.dst);
                uint8_t *d1 = d0 + pi.plen;
                uint8_t *cb = reinterpret_cast<uint8_t *>(((uintptr_t)d0 & ~(uintptr_t)15) + 16u * c);
                if (cb < d1) {
                    const uint8_t *s0 = pkts + (uint64_t)p * stride + pi.hl;
                    if (cb >= d0 && cb + 16 <= d1 && ((((uintptr_t)d0) ^ ((uintptr_t)s0)) & 3u) == 0) {
                        v[u] = ld16(s0 + (cb - d0));
                        dst[u] = cb;
                        st[u] = true;
                    } else {
                        uint8_t *lo = cb < d0 ? d0 : cb;
                        uint8_t *hi = (cb + 16 < d1) ? cb + 16 : d1;
                        copy_edge(lo, hi, s0 + (lo - d0));
                    }
                }
            }
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++)
        if (st[u]) st16(dst[u], v[u]);
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
    atomicAdd(reinterpret_cast<unsigned long long *>(&R.ctl->inProgress), ~0ull);
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

__global__ __launch_bounds__(kBlock) void reas_recycle_kernel(ReasDev R, int dropCompleted)
{
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
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
}

// ---------------------------------------------------------------------------------
// launchers

static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

hipError_t launch_segment(const e2sar_hip_seg_event *d_events, uint32_t nEvents,
                          uint32_t maxPacketsPerEvent, int lbVersion, uint32_t maxPld,
                          bool aligned4, uint8_t *pkts, uint32_t stride, uint32_t *lens,
                          hipStream_t stream)
{
    constexpr int U = 4;
    if (nEvents == 0 || maxPacketsPerEvent == 0) return hipSuccess;
    const uint64_t chunks = (uint64_t)maxPacketsPerEvent * (stride >> 4);
    const uint32_t bpe = cdiv(chunks, (uint64_t)kBlock * U);
    const uint64_t grid = (uint64_t)bpe * nEvents;
    if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
    if (aligned4)
        hipLaunchKernelGGL((seg_kernel<true, U>), dim3((uint32_t)grid), dim3(kBlock), 0, stream,
                           d_events, bpe, lbVersion, maxPld, pkts, stride, lens);
    else
        hipLaunchKernelGGL((seg_kernel<false, U>), dim3((uint32_t)grid), dim3(kBlock), 0, stream,
                           d_events, bpe, lbVersion, maxPld, pkts, stride, lens);
    return hipGetLastError();
}

hipError_t launch_reassemble(const ReasDev &R, const uint8_t *pkts, uint32_t stride,
                             const uint32_t *lens, uint32_t n, uint64_t now, PktInfo *info,
                             hipStream_t stream)
{
    constexpr int U = 4;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(reas_classify, dim3(cdiv(n, kBlock)), dim3(kBlock), 0, stream, R, pkts,
                       stride, lens, n, now, info);
    const uint32_t spc = stride >> 4;
    const uint64_t chunks = (uint64_t)n * spc;
    if (chunks > 0xFFFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL((reas_scatter<U>), dim3(cdiv(chunks, (uint64_t)kBlock * U)), dim3(kBlock), 0,
                       stream, info, pkts, stride, spc, (uint32_t)chunks);
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

}  // namespace e2sar_amd
