// ro_sort.hip -- the key sort of the reference-order reassembly mode: a stable radix sort
// of our own on the slot bits of the sort keys.
#include "sar_kernels.hpp"

namespace e2sar_amd {

// ---- slot sort: a stable LSD radix sort of the sort keys on bits [32, endBit), in 8-bit
// digits, with kernels of its own and no memset nodes (a HIP graph can hold it): per pass
// a per-tile digit histogram (digit-major), a scan of every digit's column over the tiles
// (one wave per digit), and a stable scatter whose workgroups add the digit totals' prefix
// themselves.  A tile is kSortRounds rounds of 256 keys, each round ranked with a wave
// match on the digit plus per-wave counts in LDS, so equal digits keep their input order.
namespace {
// tiles of 512 keys (256: 153.0 vs 146.9 us per batch, round 2 DESIGN 4.5)
constexpr uint32_t kSortThreads = 256, kSortRounds = 2, kSortTile = kSortThreads * kSortRounds;
constexpr uint32_t kDigits = 256;
static_assert(kSortThreads == kDigits, "one thread per digit for the per-digit LDS arrays");

__device__ __forceinline__ uint64_t digit_peers(uint32_t d, bool live)
{
    uint64_t m = __ballot(live);           // lanes of this wave holding the same 8-bit digit
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const bool bit = ((d >> b) & 1u) != 0u;
        const uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}

__global__ __launch_bounds__(kSortThreads) void slot_hist_kernel(const unsigned long long *__restrict__ in, uint32_t n,
                                                                 uint32_t shift, uint32_t mask,
                                                                 uint32_t *__restrict__ hist, uint32_t nTiles)
{
    __shared__ uint32_t c[kDigits];
    c[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
#pragma unroll
    for (uint32_t r = 0; r < kSortRounds; r++) {
        const uint64_t i = base + (uint64_t)r * kSortThreads + threadIdx.x;
        const bool live = i < n;
        const uint32_t d = live ? (uint32_t)(in[i] >> shift) & mask : 0u;
        const uint64_t peers = digit_peers(d, live);
        if (live && (peers & ((1ull << lane) - 1ull)) == 0ull) atomicAdd(&c[d], (uint32_t)__builtin_popcountll(peers));
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * nTiles + blockIdx.x] = c[threadIdx.x];
}

// One wave per digit: exclusive scan of the digit's column over the tiles, in place; the
// column's total to totals[d].
__global__ __launch_bounds__(kSortThreads) void slot_colscan_kernel(uint32_t *__restrict__ hist, uint32_t nTiles,
                                                                    uint32_t *__restrict__ totals)
{
    const uint32_t d = blockIdx.x * (kSortThreads / 64u) + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (d >= kDigits) return;
    uint32_t *col = hist + (uint64_t)d * nTiles;
    uint32_t carry = 0;
    for (uint32_t t0 = 0; t0 < nTiles; t0 += 64u) {
        const uint32_t t = t0 + lane;
        const uint32_t v = (t < nTiles) ? col[t] : 0u;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o);
            if ((int)lane >= o) x += y;
        }
        if (t < nTiles) col[t] = carry + x - v;
        carry += (uint32_t)__shfl((int)x, 63);
    }
    if (lane == 0) totals[d] = carry;
}

__global__ __launch_bounds__(kSortThreads) void slot_scatter_kernel(const unsigned long long *__restrict__ in,
                                                                    unsigned long long *__restrict__ out, uint32_t n,
                                                                    uint32_t shift, uint32_t mask,
                                                                    const uint32_t *__restrict__ hist,
                                                                    const uint32_t *__restrict__ totals, uint32_t nTiles)
{
    __shared__ uint32_t pos0[kDigits];            // next output position of each digit for this tile
    __shared__ uint32_t sc[kDigits];
    __shared__ uint32_t wc[kSortThreads / 64][kDigits];
    const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
    // digit bases: exclusive prefix of the totals (every workgroup, 256 entries)
    const uint32_t tot = totals[t];
    sc[t] = tot;
    __syncthreads();
    for (uint32_t off = 1; off < kDigits; off <<= 1) {
        const uint32_t v = (t >= off) ? sc[t - off] : 0u;
        __syncthreads();
        sc[t] += v;
        __syncthreads();
    }
    pos0[t] = sc[t] - tot + hist[(uint64_t)t * nTiles + blockIdx.x];
    const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
    for (uint32_t r = 0; r < kSortRounds; r++) {
#pragma unroll
        for (uint32_t w = 0; w < kSortThreads / 64; w++) wc[w][t] = 0u;
        __syncthreads();
        const uint64_t i = base + (uint64_t)r * kSortThreads + t;
        const bool live = i < n;
        const unsigned long long k = live ? in[i] : 0ull;
        const uint32_t d = live ? (uint32_t)(k >> shift) & mask : 0u;
        const uint64_t peers = digit_peers(d, live);
        const uint32_t rank = (uint32_t)__builtin_popcountll(peers & ((1ull << lane) - 1ull));
        if (live && rank == 0u) wc[wave][d] = (uint32_t)__builtin_popcountll(peers);
        __syncthreads();
        if (live) {
            uint32_t before = 0;
            for (uint32_t w = 0; w < wave; w++) before += wc[w][d];
            out[pos0[d] + before + rank] = k;
        }
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (uint32_t w = 0; w < kSortThreads / 64; w++) add += wc[w][t];
        pos0[t] += add;
    }
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

hipError_t slot_sort(void *temp, size_t &tempBytes, const unsigned long long *in, unsigned long long *out, uint32_t n,
                     unsigned endBit, hipStream_t stream)
{
    const uint32_t nTiles = (n + kSortTile - 1u) / kSortTile;
    const uint32_t bits = endBit > 32u ? endBit - 32u : 0u;
    const uint32_t passes = (bits + 7u) / 8u;
    const size_t histB = align256((size_t)4 * kDigits * (nTiles ? nTiles : 1u));
    const size_t totB = align256((size_t)4 * kDigits);
    const size_t tmpB = passes > 1u ? align256((size_t)8 * n) : 0u;
    if (!temp) {
        tempBytes = histB + totB + tmpB;
        return hipSuccess;
    }
    if (tempBytes < histB + totB + tmpB) return hipErrorInvalidValue;
    if (n == 0u) return hipSuccess;
    if (passes == 0u) return hipMemcpyAsync(out, in, (size_t)8 * n, hipMemcpyDeviceToDevice, stream);   // copy node: replays clean
    uint8_t *tb = static_cast<uint8_t *>(temp);
    uint32_t *hist = reinterpret_cast<uint32_t *>(tb);
    uint32_t *totals = reinterpret_cast<uint32_t *>(tb + histB);
    unsigned long long *tmp = reinterpret_cast<unsigned long long *>(tb + histB + totB);
    const unsigned long long *src = in;
    for (uint32_t p = 0; p < passes; p++) {
        const uint32_t shift = 32u + 8u * p;
        const uint32_t nb = (bits - 8u * p < 8u) ? bits - 8u * p : 8u;
        const uint32_t mask = (1u << nb) - 1u;
        unsigned long long *dst = ((passes - 1u - p) % 2u == 0u) ? out : tmp;   // the last pass lands in out
        hipLaunchKernelGGL(slot_hist_kernel, dim3(nTiles), dim3(kSortThreads), 0, stream, src, n, shift, mask, hist,
                           nTiles);
        hipLaunchKernelGGL(slot_colscan_kernel, dim3(kDigits / (kSortThreads / 64u)), dim3(kSortThreads), 0, stream,
                           hist, nTiles, totals);
        hipLaunchKernelGGL(slot_scatter_kernel, dim3(nTiles), dim3(kSortThreads), 0, stream, src, dst, n, shift, mask,
                           hist, totals, nTiles);
        src = dst;
    }
    return hipGetLastError();
}
}  // namespace

hipError_t ro_sort_keys(void *temp, size_t &tempBytes, const unsigned long long *in, unsigned long long *out,
                        uint32_t n, unsigned endBit, hipStream_t stream)
{
    // keys are slot << 32 | position and arrive in position order; the sort is stable, so
    // sorting the slot bits alone (32 .. endBit) keeps each slot's positions in order.
    // The slot sort above: 6 launches for 14 bits, 147.2 us per 205-event batch against
    // 179.5 with rocPRIM's merge-sort form (9 launches) and 162.4 with its onesweep form
    // (round 2 A/B).  rocPRIM is not used: its onesweep form memsets look-back
    // states, and a captured memset node writes garbage from the second replay on (DESIGN.md
    // 4.4), so only a sort without memset nodes may run where a caller can capture.
    return slot_sort(temp, tempBytes, in, out, n, endBit, stream);
}

size_t ro_scratch_bytes(uint32_t n, uint32_t tableSlots)
{
    size_t tb = 0;
    if (ro_sort_keys(nullptr, tb, nullptr, nullptr, n, ro_sort_end_bit(tableSlots), nullptr) != hipSuccess) return 0;
    return ro_fixed_bytes(n) + ro_align(tb);
}

}  // namespace e2sar_amd
