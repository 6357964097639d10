// ubench_rounds.hip -- why do multi-round copy workgroups run slower than one-round ones on
// the reassembly's data (the scatter at 49 datagrams per workgroup 74.4 us,
// at 8 datagrams 68.2 us)?  Kernel W writes `mid` from uniform random `src` (8-KiB pieces,
// plain stores, as seg_kernel does); kernel R copies mid -> dst (16-B loads, non-temporal
// 16-B stores), every workgroup 256 threads moving R rounds of 16 KiB (4 chunks per thread
// per round), in one of these forms:
//   one    : R = 1 (one-round workgroups, the scatter's shape)
//   naive  : per round load 4, store 4 (a round's loads wait for the previous stores' acks:
//            vmcnt retires loads and stores in issue order)
//   pipe   : loads of round r+1 issued before the stores of round r (the fused kernel's loop)
//   all    : every round's loads issued first (R x 4 chunks per thread in registers), then
//            every store: no load ever waits behind a store
//   spec   : 512-thread workgroups, waves 0-3 load (global_load_lds into an LDS ring of 4
//            16-KiB slots), waves 4-7 read the ring and store: the storing waves never load
//            from memory, the loading waves never store
// Only R is timed (HIP events around it, median of iterations).
// Usage: ubench_rounds [MiB] [iters] -> one JSON line (us)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GA __attribute__((address_space(1)))

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const GA u32x4 *)p); }
__device__ __forceinline__ u32x4 ld(const uint8_t *p) { return *(const GA u32x4 *)p; }
__device__ __forceinline__ void stnt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (GA u32x4 *)p); }

__global__ __launch_bounds__(256) void fill_random(uint8_t *p, uint64_t n16, uint64_t seed)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        uint64_t y = z * 0xD6E8FEB86659FD93ull;
        y ^= y >> 32;
        *(GA u32x4 *)(p + 16 * i) = u32x4{(uint32_t)z, (uint32_t)(z >> 32), (uint32_t)y, (uint32_t)(y >> 32)};
    }
}

__global__ __launch_bounds__(256) void wk(const uint8_t *src, uint8_t *mid)
{
    const uint64_t base = (uint64_t)blockIdx.x * 8192;
    u32x4 v[2];
#pragma unroll
    for (int u = 0; u < 2; u++) v[u] = ldnt(src + base + (u * 256 + threadIdx.x) * 16);
#pragma unroll
    for (int u = 0; u < 2; u++) *(GA u32x4 *)(mid + base + (u * 256 + threadIdx.x) * 16) = v[u];
}

template <int R>
__global__ __launch_bounds__(256) void rk_naive(const uint8_t *mid, uint8_t *dst)
{
    const uint64_t base = (uint64_t)blockIdx.x * R * 16384;
    for (int r = 0; r < R; r++) {
        u32x4 v[4];
        const uint64_t o = base + (uint64_t)r * 16384;
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = ld(mid + o + (u * 256 + threadIdx.x) * 16);
#pragma unroll
        for (int u = 0; u < 4; u++) stnt(dst + o + (u * 256 + threadIdx.x) * 16, v[u]);
    }
}

template <int R>
__global__ __launch_bounds__(256) void rk_pipe(const uint8_t *mid, uint8_t *dst)
{
    const uint64_t base = (uint64_t)blockIdx.x * R * 16384;
    u32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; u++) x[u] = ld(mid + base + (u * 256 + threadIdx.x) * 16);
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint64_t o = base + (uint64_t)r * 16384;
        if (r + 1 < R) {
#pragma unroll
            for (int u = 0; u < 4; u++) y[u] = ld(mid + o + 16384 + (u * 256 + threadIdx.x) * 16);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) stnt(dst + o + (u * 256 + threadIdx.x) * 16, x[u]);
#pragma unroll
        for (int u = 0; u < 4; u++) x[u] = y[u];
    }
}

template <int R>
__global__ __launch_bounds__(256) void rk_all(const uint8_t *mid, uint8_t *dst)
{
    const uint64_t base = (uint64_t)blockIdx.x * R * 16384;
    u32x4 v[R * 4];
#pragma unroll
    for (int k = 0; k < R * 4; k++) v[k] = ld(mid + base + (k * 256 + threadIdx.x) * 16);
#pragma unroll
    for (int k = 0; k < R * 4; k++) stnt(dst + base + (k * 256 + threadIdx.x) * 16, v[k]);
}

// Warp-specialised: 8 waves; waves 0-3 fill LDS ring slots with global_load_lds (16 B per
// lane per instruction), waves 4-7 drain them with ds_read_b128 + nt stores.  One s_barrier
// per round hands a slot over (loaders are kSlots-1 rounds ahead).
constexpr int kSlots = 4;
template <int R>
__global__ __launch_bounds__(512) void rk_spec(const uint8_t *mid, uint8_t *dst)
{
    __shared__ __attribute__((aligned(16))) uint8_t ring[kSlots][16384];
    const uint64_t base = (uint64_t)blockIdx.x * R * 16384;
    const uint32_t t = threadIdx.x;
    const bool loader = t < 256;
    const uint32_t lt = t & 255u;
    auto fill = [&](int r) {
        // 4 chunks per loader thread: chunk u*256 + lt of round r into ring slot r % kSlots
        uint8_t *slot = ring[r % kSlots];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint8_t *g = mid + base + (uint64_t)r * 16384 + (u * 256 + lt) * 16;
            // LDS destination: M0 = wave's base in the slot; each lane writes 16 B at
            // M0 + lane*16 (global_load_lds_dwordx4)
            __builtin_amdgcn_global_load_lds((const GA void *)g,
                                             (__attribute__((address_space(3))) void *)(slot + (u * 256 + (lt & ~63u)) * 16),
                                             16, 0, 0);
        }
    };
    if (loader) {
        for (int r = 0; r < kSlots - 1 && r < R; r++) fill(r);
    }
    for (int r = 0; r < R; r++) {
        if (loader) {
            if (r + kSlots - 1 < R) {
                fill(r + kSlots - 1);
                // round r's fills are the oldest kSlots-1 groups of 4 in flight
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (kSlots - 1)) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __builtin_amdgcn_s_barrier();
        if (!loader) {
            const uint8_t *slot = ring[r % kSlots];
            u32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = *(const __attribute__((address_space(3))) u32x4 *)(slot + (u * 256 + lt) * 16);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int u = 0; u < 4; u++) stnt(dst + base + (uint64_t)r * 16384 + (u * 256 + lt) * 16, v[u]);
        }
        __builtin_amdgcn_s_barrier();       // slot r % kSlots read: loaders may refill it
    }
}

// ---- datagram-shaped copies: the reassembly's access pattern without classification ----
// Slots of 1472 B (36-B headers, 1436-B payloads) -> one contiguous event (datagram p's
// payload at p x 1436), destination-aligned as reas_kernel: chunk c of datagram p covers
// event bytes [(p x 1436 & ~15) + 16c, +16), loaded from the slot at 36 + 16c - a (a = the
// payload's phase, dword aligned), slid back inside the slot at its end; whole chunks stored
// aligned, the two edges as dword stores.  Workgroup g copies datagrams [gG, gG + G) in
// rounds of 1024 chunks (92 chunk slots per datagram, as the fused kernel indexes them).
constexpr uint32_t kStride = 1472, kHl = 36, kPl = 1436, kSpc = kStride / 16;

struct DgChunk {
    uint32_t p, c;
    bool live;
};
__device__ __forceinline__ DgChunk dg_split(uint32_t i, uint32_t nch)
{
    DgChunk d;
    d.live = i < nch;
    const uint32_t ic = d.live ? i : 0u;
    d.p = ic / kSpc;
    d.c = ic - d.p * kSpc;
    return d;
}
__device__ __forceinline__ u32x4 dg_load(const uint8_t *slots, uint32_t pg, DgChunk d)
{
    const uint32_t a = ((pg + d.p) * kPl) & 15u;
    uint32_t off = 0;
    if (d.live && 16u * d.c < a + kPl) {
        uint32_t r = kHl + 16u * d.c - a;
        if (r + 16u > kStride) r = kStride - 16u;
        off = d.p * kStride + r;
    }
    return *(const GA u32x4 *)(slots + off);
}
__device__ __forceinline__ void dg_store(uint8_t *dst, uint32_t pg, DgChunk d, u32x4 x)
{
    if (!d.live) return;
    const uint32_t P = pg + d.p;
    const uint32_t a = (P * kPl) & 15u;
    if (16u * d.c >= a + kPl) return;
    uint32_t r = kHl + 16u * d.c - a, sh = 0;
    if (r + 16u > kStride) sh = (r + 16u - kStride) >> 2;
    u32x4 o = x;
    if (sh == 1) o = u32x4{x.y, x.z, x.w, 0u};
    else if (sh == 2) o = u32x4{x.z, x.w, 0u, 0u};
    else if (sh == 3) o = u32x4{x.w, 0u, 0u, 0u};
    uint8_t *D = dst + (((uint64_t)P * kPl) & ~15ull) + 16ull * d.c;
    const uint32_t lo = d.c == 0 ? a : 0u;
    const uint32_t hi = (a + kPl - 16u * d.c < 16u) ? a + kPl - 16u * d.c : 16u;
    if (lo == 0 && hi == 16) {
        stnt(D, o);
    } else {
        for (uint32_t w = lo / 4; w < hi / 4; w++) *(GA uint32_t *)(D + 4 * w) = o[w];
    }
}

template <int G>
__global__ __launch_bounds__(256) void dg_naive(const uint8_t *slots, uint8_t *dst, uint32_t n)
{
    const uint32_t pg = blockIdx.x * G;
    const uint32_t gn = (n - pg < G) ? n - pg : G;
    const uint32_t nch = gn * kSpc;
    const uint8_t *s = slots + (uint64_t)pg * kStride;
    for (uint32_t r0 = 0; r0 < nch; r0 += 1024) {
        u32x4 x[4];
        DgChunk d[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            d[u] = dg_split(r0 + u * 256 + threadIdx.x, nch);
            x[u] = dg_load(s, pg, d[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) dg_store(dst, pg, d[u], x[u]);
    }
}

// rounds aligned to datagram boundaries: round k covers datagrams [11k, 11k + 11) (1012 of
// 1024 lanes), so no datagram straddles two rounds
template <int G>
__global__ __launch_bounds__(256) void dg_rows(const uint8_t *slots, uint8_t *dst, uint32_t n)
{
    const uint32_t pg = blockIdx.x * G;
    const uint32_t gn = (n - pg < G) ? n - pg : G;
    const uint8_t *s = slots + (uint64_t)pg * kStride;
    for (uint32_t q0 = 0; q0 < gn; q0 += 11) {
        const uint32_t qn = (gn - q0 < 11) ? gn - q0 : 11;
        const uint32_t nch = qn * kSpc;
        u32x4 x[4];
        DgChunk d[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            d[u] = dg_split(u * 256 + threadIdx.x, nch);
            d[u].p += q0;
            x[u] = dg_load(s, pg, d[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) dg_store(dst, pg, d[u], x[u]);
    }
}

template <int G>
__global__ __launch_bounds__(256) void dg_pipe(const uint8_t *slots, uint8_t *dst, uint32_t n)
{
    const uint32_t pg = blockIdx.x * G;
    const uint32_t gn = (n - pg < G) ? n - pg : G;
    const uint32_t nch = gn * kSpc;
    const uint8_t *s = slots + (uint64_t)pg * kStride;
    u32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; u++) x[u] = dg_load(s, pg, dg_split(u * 256 + threadIdx.x, nch));
    for (uint32_t r0 = 0; r0 < nch; r0 += 1024) {
        if (r0 + 1024 < nch) {
#pragma unroll
            for (int u = 0; u < 4; u++) y[u] = dg_load(s, pg, dg_split(r0 + 1024 + u * 256 + threadIdx.x, nch));
        }
#pragma unroll
        for (int u = 0; u < 4; u++) dg_store(dst, pg, dg_split(r0 + u * 256 + threadIdx.x, nch), x[u]);
#pragma unroll
        for (int u = 0; u < 4; u++) x[u] = y[u];
    }
}

template <int G, int R>
__global__ __launch_bounds__(256) void dg_all(const uint8_t *slots, uint8_t *dst, uint32_t n)
{
    const uint32_t pg = blockIdx.x * G;
    const uint32_t gn = (n - pg < G) ? n - pg : G;
    const uint32_t nch = gn * kSpc;
    const uint8_t *s = slots + (uint64_t)pg * kStride;
    u32x4 x[R * 4];
#pragma unroll
    for (int k = 0; k < R * 4; k++) x[k] = dg_load(s, pg, dg_split(k * 256 + threadIdx.x, nch));
#pragma unroll
    for (int k = 0; k < R * 4; k++) dg_store(dst, pg, dg_split(k * 256 + threadIdx.x, nch), x[k]);
}

// dg_pipe<49> plus the fused kernel's non-copy parts, one at a time (MODE bits):
//   1: wave 0 writes every datagram's destination to LDS, barrier, stores read it from LDS
//   2: wave 0 waits SLEEP_US (s_memrealtime) before that barrier -- a classification's
//      latency -- with round 0's loads in flight
//   4: each run tail (here: lane 0 of wave 0) issues a returning atomic add on its event's
//      counter (event = datagram / 731) before round 1's loads; its result is used last
struct MockLds {
    uint64_t dst[64];
};
template <int G, int MODE>
__global__ __launch_bounds__(256) void dg_mock(const uint8_t *slots, uint8_t *dst, uint32_t n,
                                               unsigned long long *ctr, uint32_t sleepTicks)
{
    __shared__ MockLds L;
    const uint32_t pg = blockIdx.x * G;
    const uint32_t gn = (n - pg < G) ? n - pg : G;
    const uint32_t nch = gn * kSpc;
    const uint8_t *s = slots + (uint64_t)pg * kStride;
    u32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; u++) x[u] = dg_load(s, pg, dg_split(u * 256 + threadIdx.x, nch));
    unsigned long long old = 0;
    if (threadIdx.x < 64) {
        if (MODE & 2) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < sleepTicks) __builtin_amdgcn_s_sleep(8);
        }
        if ((MODE & 4) && threadIdx.x == 0) old = atomicAdd(ctr + (pg / 731u) * 16u, 1ull);
        if (MODE & 1) L.dst[threadIdx.x] = (uint64_t)(dst) + (uint64_t)(pg + threadIdx.x) * kPl;
    }
    if (MODE & 3) __syncthreads();
    for (uint32_t r0 = 0; r0 < nch; r0 += 1024) {
        if (r0 + 1024 < nch) {
#pragma unroll
            for (int u = 0; u < 4; u++) y[u] = dg_load(s, pg, dg_split(r0 + 1024 + u * 256 + threadIdx.x, nch));
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const DgChunk d = dg_split(r0 + u * 256 + threadIdx.x, nch);
            uint8_t *D = dst;
            if (MODE & 1) D = reinterpret_cast<uint8_t *>(L.dst[d.p]) - (uint64_t)(pg + d.p) * kPl;
            dg_store(D, pg, d, x[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) x[u] = y[u];
    }
    if ((MODE & 4) && threadIdx.x == 0 && old == ~0ull) ctr[1] = 1;      // consume the result
}

__global__ __launch_bounds__(256) void wk_slots(const uint8_t *src, uint8_t *slots, uint32_t n)
{
    // seg-shaped writer: 8-KiB pieces of the slot array from a random source
    const uint64_t base = (uint64_t)blockIdx.x * 8192;
    const uint64_t lim = (uint64_t)n * kStride;
    u32x4 v[2];
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const uint64_t o = base + (u * 256 + threadIdx.x) * 16;
        v[u] = o < lim ? ldnt(src + o) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const uint64_t o = base + (u * 256 + threadIdx.x) * 16;
        if (o < lim) *(GA u32x4 *)(slots + o) = v[u];
    }
}

int main(int argc, char **argv)
{
    const uint64_t mib = argc > 1 ? atoll(argv[1]) : 210;
    const int iters = argc > 2 ? atoi(argv[2]) : 15;
    const uint64_t unit = 16384ull * 40;              // divisible by every R below (1, 4, 5, 8)
    const uint64_t bytes = (mib << 20) / unit * unit;
    uint8_t *src, *mid, *dst;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&mid, bytes));
    CHECK(hipMalloc(&dst, bytes));
    fill_random<<<4096, 256>>>(src, bytes / 16, 12345);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto timeit = [&](auto launch) {
        std::vector<float> v;
        for (int i = 0; i < iters; i++) {
            wk<<<bytes / 8192, 256>>>(src, mid);
            CHECK(hipEventRecord(a));
            launch();
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            v.push_back(ms * 1000.0f);
        }
        CHECK(hipGetLastError());
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
#define NWG(R) (unsigned)(bytes / (16384ull * (R)))
    printf("{\"MiB\": %llu", (unsigned long long)(bytes >> 20));
    for (int rep = 0; rep < 2; rep++) {
        printf(", \"rep%d\": {", rep);
        printf("\"one\": %.2f", timeit([&] { rk_naive<1><<<NWG(1), 256>>>(mid, dst); }));
        printf(", \"naive4\": %.2f", timeit([&] { rk_naive<4><<<NWG(4), 256>>>(mid, dst); }));
        printf(", \"naive5\": %.2f", timeit([&] { rk_naive<5><<<NWG(5), 256>>>(mid, dst); }));
        printf(", \"pipe5\": %.2f", timeit([&] { rk_pipe<5><<<NWG(5), 256>>>(mid, dst); }));
        printf(", \"pipe8\": %.2f", timeit([&] { rk_pipe<8><<<NWG(8), 256>>>(mid, dst); }));
        printf(", \"all4\": %.2f", timeit([&] { rk_all<4><<<NWG(4), 256>>>(mid, dst); }));
        printf(", \"all5\": %.2f", timeit([&] { rk_all<5><<<NWG(5), 256>>>(mid, dst); }));
        printf(", \"spec5\": %.2f", timeit([&] { rk_spec<5><<<NWG(5), 512>>>(mid, dst); }));
        printf(", \"spec8\": %.2f", timeit([&] { rk_spec<8><<<NWG(8), 512>>>(mid, dst); }));
        printf("}");
    }
    // datagram-shaped: 146,165 datagrams (205 x 1 MiB events at MTU 1500) = 215 MB of slots
    const uint32_t n = 146165;
    uint8_t *slots;
    CHECK(hipMalloc(&slots, (uint64_t)n * kStride + 4096));
    unsigned long long *ctr;
    CHECK(hipMalloc(&ctr, 1 << 20));
    CHECK(hipMemset(ctr, 0, 1 << 20));
    auto timedg = [&](auto launch) {
        std::vector<float> v;
        for (int i = 0; i < iters; i++) {
            wk_slots<<<(unsigned)(((uint64_t)n * kStride + 8191) / 8192), 256>>>(src, slots, n);
            CHECK(hipEventRecord(a));
            launch();
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            v.push_back(ms * 1000.0f);
        }
        CHECK(hipGetLastError());
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
#define NG(G) (unsigned)((n + (G) - 1) / (G))
    for (int rep = 0; rep < 2; rep++) {
        printf(", \"dg_rep%d\": {", rep);
        printf("\"one8\": %.2f", timedg([&] { dg_naive<8><<<NG(8), 256>>>(slots, dst, n); }));
        printf(", \"one11\": %.2f", timedg([&] { dg_naive<11><<<NG(11), 256>>>(slots, dst, n); }));
        printf(", \"naive49\": %.2f", timedg([&] { dg_naive<49><<<NG(49), 256>>>(slots, dst, n); }));
        printf(", \"pipe49\": %.2f", timedg([&] { dg_pipe<49><<<NG(49), 256>>>(slots, dst, n); }));
        printf(", \"all49\": %.2f", timedg([&] { dg_all<49, 5><<<NG(49), 256>>>(slots, dst, n); }));
        printf(", \"all33\": %.2f", timedg([&] { dg_all<33, 3><<<NG(33), 256>>>(slots, dst, n); }));
        printf(", \"pipe22\": %.2f", timedg([&] { dg_pipe<22><<<NG(22), 256>>>(slots, dst, n); }));
        printf(", \"naive16\": %.2f", timedg([&] { dg_naive<16><<<NG(16), 256>>>(slots, dst, n); }));
        printf(", \"naive24\": %.2f", timedg([&] { dg_naive<24><<<NG(24), 256>>>(slots, dst, n); }));
        printf(", \"naive32\": %.2f", timedg([&] { dg_naive<32><<<NG(32), 256>>>(slots, dst, n); }));
        printf(", \"rows44\": %.2f", timedg([&] { dg_rows<44><<<NG(44), 256>>>(slots, dst, n); }));
        printf(", \"rows22\": %.2f", timedg([&] { dg_rows<22><<<NG(22), 256>>>(slots, dst, n); }));
        printf(", \"mock_lds\": %.2f", timedg([&] { dg_mock<49, 1><<<NG(49), 256>>>(slots, dst, n, ctr, 0); }));
        printf(", \"mock_sleep3\": %.2f", timedg([&] { dg_mock<49, 3><<<NG(49), 256>>>(slots, dst, n, ctr, 300); }));
        printf(", \"mock_sleep7\": %.2f", timedg([&] { dg_mock<49, 3><<<NG(49), 256>>>(slots, dst, n, ctr, 700); }));
        printf(", \"mock_atomic\": %.2f", timedg([&] { dg_mock<49, 4><<<NG(49), 256>>>(slots, dst, n, ctr, 0); }));
        printf(", \"mock_all7\": %.2f", timedg([&] { dg_mock<49, 7><<<NG(49), 256>>>(slots, dst, n, ctr, 700); }));
        // the fused kernel's residency (6 workgroups per CU): 24 KiB of dynamic LDS each
        printf(", \"one8_occ6\": %.2f", timedg([&] { dg_naive<8><<<NG(8), 256, 24576>>>(slots, dst, n); }));
        printf(", \"pipe49_occ6\": %.2f", timedg([&] { dg_pipe<49><<<NG(49), 256, 24576>>>(slots, dst, n); }));
        printf("}");
    }
    printf("}\n");
    return 0;
}
