// ubench_slab.hip -- can a reassembly workgroup take its whole group of datagrams into LDS
// (global_load_lds, no VGPRs held) while its classification runs, and then store, at the
// speed of a one-round copy?  DESIGN.md 4.5: the fused kernel's 75 us against the 66 us of a
// one-round copy are ~4.5 us of multi-round, datagram-shaped workgroups and ~4 us of a
// ~7 us classification stall that only the round-0 loads (held in VGPRs) cover.
//
// Same data as ubench_rounds' datagram forms: 146,165 slots of 1472 B (36-B headers,
// 1436-B payloads) written by a seg-shaped kernel, copied into one contiguous destination
// (datagram p's payload at p x 1436).  Kernel slab<G, NT, MODE>, workgroup = G datagrams:
//   1. every wave issues global_load_lds_dwordx4 for its share of the group's slot bytes
//      (one linear copy of G x 1472 B into LDS);
//   2. MODE & 4: wave 0 then waits SLEEP ticks (a mocked classification);
//   3. s_waitcnt vmcnt(0) + barrier;
//   4. stores: MODE & 1 == 0: per datagram, destination-aligned 16-B chunks (the fused
//      kernel's store pattern, edges as dword stores); MODE & 1: per run (the group's
//      datagrams are one contiguous destination range), aligned 16-B chunks over the whole
//      range, each dword read from the datagram that holds it -- edge stores only at the
//      run's two ends.
// Usage: ubench_slab [iters] -> one JSON line (us, median)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GA __attribute__((address_space(1)))
#define LA __attribute__((address_space(3)))

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const GA u32x4 *)p); }
__device__ __forceinline__ void stnt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (GA u32x4 *)p); }

constexpr uint32_t kStride = 1472, kHl = 36, kPl = 1436, kSpc = kStride / 16;

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

__global__ __launch_bounds__(256) void wk_slots(const uint8_t *src, uint8_t *slots, uint32_t n)
{
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

__device__ __forceinline__ u32x4 lds16(const uint8_t *slab, uint32_t r)
{
    const LA uint32_t *w = (const LA uint32_t *)(slab + r);
    return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ void store_edge(uint8_t *D, u32x4 o, uint32_t lo, uint32_t hi)
{
    for (uint32_t w = lo / 4; w < hi / 4; w++) *(GA uint32_t *)(D + 4 * w) = o[w];
}

template <int G, int NT, int MODE>
__global__ __launch_bounds__(NT) void slab(const uint8_t *slots, uint8_t *dst, uint32_t n, uint32_t sleepTicks)
{
    __shared__ __attribute__((aligned(16))) uint8_t S[G * kStride + 64];
    const uint32_t pg = blockIdx.x * G;
    const uint32_t gn = (n - pg < G) ? n - pg : G;
    const uint32_t nc = gn * kSpc;                     // 16-B chunks of the group's slots
    const uint8_t *s = slots + (uint64_t)pg * kStride;
    const uint32_t tx = threadIdx.x, lane = tx & 63u, wv = tx >> 6;
    constexpr uint32_t W = NT / 64;
    for (uint32_t k = wv; k * 64u < nc; k += W) {
        const uint32_t c = k * 64u + lane;
        if (c < nc)
            __builtin_amdgcn_global_load_lds((const GA void *)(s + 16ull * c), (LA void *)(S + 1024u * k), 16, 0, 0);
    }
    if ((MODE & 4) && wv == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < sleepTicks) __builtin_amdgcn_s_sleep(8);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if ((MODE & 1) == 0) {
        // per datagram: chunk c of datagram p covers destination [(P*1436 & ~15) + 16c, +16)
        for (uint32_t i = tx; i < nc; i += NT) {
            const uint32_t p = i / kSpc, c = i - p * kSpc;
            const uint32_t P = pg + p;
            const uint32_t a = (P * kPl) & 15u;
            if (16u * c >= a + kPl) continue;
            const u32x4 x = lds16(S, p * kStride + kHl + 16u * c - a);
            uint8_t *D = dst + (((uint64_t)P * kPl) & ~15ull) + 16ull * c;
            const uint32_t lo = c == 0 ? a : 0u;
            const uint32_t hi = (a + kPl - 16u * c < 16u) ? a + kPl - 16u * c : 16u;
            if (lo == 0 && hi == 16) stnt(D, x);
            else store_edge(D, x, lo, hi);
        }
    } else {
        // per run: the group's destination [D0, D1) in aligned 16-B chunks
        const uint64_t D0 = (uint64_t)pg * kPl, D1 = D0 + (uint64_t)gn * kPl;
        const uint64_t A0 = D0 & ~15ull;
        const uint32_t nk = (uint32_t)(((D1 + 15u) & ~15ull) - A0) >> 4;
        for (uint32_t k = tx; k < nk; k += NT) {
            const uint64_t e0 = A0 + 16ull * k;
            // first dword at or after D0
            const uint32_t lo = (e0 < D0) ? (uint32_t)(D0 - e0) : 0u;
            const uint32_t hi = (e0 + 16u > D1) ? (uint32_t)(D1 - e0) : 16u;
            uint32_t rel = (uint32_t)(e0 + lo - D0);
            uint32_t q = rel / kPl, r = rel - q * kPl;
            u32x4 o = {0, 0, 0, 0};
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                if (4u * j >= lo && 4u * j < hi) {
                    o[j] = *(const LA uint32_t *)(S + q * kStride + kHl + r);
                    r += 4u;
                    if (r == kPl) { r = 0; q++; }
                }
            }
            uint8_t *D = dst + e0;
            if (lo == 0 && hi == 16) stnt(D, o);
            else store_edge(D, o, lo, hi);
        }
    }
}

// reference point: the one-round 8-datagram register copy of ubench_rounds (dg_naive<8>)
__global__ __launch_bounds__(256) void one8(const uint8_t *slots, uint8_t *dst, uint32_t n)
{
    const uint32_t pg = blockIdx.x * 8;
    const uint32_t gn = (n - pg < 8) ? n - pg : 8;
    const uint32_t nch = gn * kSpc;
    const uint8_t *s = slots + (uint64_t)pg * kStride;
    u32x4 x[4];
    uint32_t pp[4], cc[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t i = u * 256 + threadIdx.x;
        const uint32_t ic = i < nch ? i : 0u;
        pp[u] = ic / kSpc;
        cc[u] = ic - pp[u] * kSpc;
        const uint32_t a = ((pg + pp[u]) * kPl) & 15u;
        uint32_t off = 0;
        if (i < nch && 16u * cc[u] < a + kPl) {
            uint32_t r = kHl + 16u * cc[u] - a;
            if (r + 16u > kStride) r = kStride - 16u;
            off = pp[u] * kStride + r;
        }
        x[u] = *(const GA u32x4 *)(s + off);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t i = u * 256 + threadIdx.x;
        if (i >= nch) continue;
        const uint32_t P = pg + pp[u], c = cc[u];
        const uint32_t a = (P * kPl) & 15u;
        if (16u * c >= a + kPl) continue;
        uint32_t r = kHl + 16u * c - a, sh = 0;
        if (r + 16u > kStride) sh = (r + 16u - kStride) >> 2;
        u32x4 o = x[u];
        if (sh == 1) o = u32x4{o.y, o.z, o.w, 0u};
        else if (sh == 2) o = u32x4{o.z, o.w, 0u, 0u};
        else if (sh == 3) o = u32x4{o.w, 0u, 0u, 0u};
        uint8_t *D = dst + (((uint64_t)P * kPl) & ~15ull) + 16ull * c;
        const uint32_t lo = c == 0 ? a : 0u;
        const uint32_t hi = (a + kPl - 16u * c < 16u) ? a + kPl - 16u * c : 16u;
        if (lo == 0 && hi == 16) stnt(D, o);
        else store_edge(D, o, lo, hi);
    }
}

__global__ void cmp_kernel(const uint8_t *a, const uint8_t *b, uint64_t n, unsigned long long *bad)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (a[i] != b[i]) atomicAdd(bad, 1ull);
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 15;
    const uint32_t n = 146165;
    const uint64_t sbytes = (uint64_t)n * kStride, dbytes = (uint64_t)n * kPl;
    uint8_t *src, *slots, *dst, *ref;
    CHECK(hipMalloc(&src, sbytes + 8192));
    CHECK(hipMalloc(&slots, sbytes + 8192));
    CHECK(hipMalloc(&dst, dbytes + 4096));
    CHECK(hipMalloc(&ref, dbytes + 4096));
    unsigned long long *bad;
    CHECK(hipMalloc(&bad, 8));
    fill_random<<<4096, 256>>>(src, (sbytes + 8192) / 16, 12345);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const unsigned wgw = (unsigned)((sbytes + 8191) / 8192);
    // reference result
    wk_slots<<<wgw, 256>>>(src, slots, n);
    one8<<<(n + 7) / 8, 256>>>(slots, ref, n);
    CHECK(hipDeviceSynchronize());
    auto timeit = [&](const char *name, auto launch) {
        std::vector<float> v;
        for (int i = 0; i < iters; i++) {
            wk_slots<<<wgw, 256>>>(src, slots, n);
            CHECK(hipEventRecord(a));
            launch();
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            v.push_back(ms * 1000.0f);
        }
        CHECK(hipGetLastError());
        CHECK(hipMemset(bad, 0, 8));
        cmp_kernel<<<2048, 256>>>(dst, ref, dbytes, bad);
        unsigned long long hb = 0;
        CHECK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
        CHECK(hipMemset(dst, 0, dbytes));
        std::sort(v.begin(), v.end());
        printf("%s\"%s\": %.2f%s", name[0] == '!' ? "" : ", ", name + (name[0] == '!'), v[v.size() / 2],
               hb ? "/*MISMATCH*/" : "");
        if (hb) fprintf(stderr, "%s: %llu bytes differ\n", name, hb);
    };
#define NG(G) (unsigned)((n + (G) - 1) / (G))
    printf("{");
    for (int rep = 0; rep < 2; rep++) {
        printf("%s\"rep%d\": {", rep ? ", " : "", rep);
        timeit("!one8", [&] { one8<<<NG(8), 256>>>(slots, dst, n); });
        timeit("slab49_t256_dg", [&] { slab<49, 256, 0><<<NG(49), 256>>>(slots, dst, n, 0); });
        timeit("slab49_t256_run", [&] { slab<49, 256, 1><<<NG(49), 256>>>(slots, dst, n, 0); });
        timeit("slab49_t512_dg", [&] { slab<49, 512, 0><<<NG(49), 512>>>(slots, dst, n, 0); });
        timeit("slab49_t512_run", [&] { slab<49, 512, 1><<<NG(49), 512>>>(slots, dst, n, 0); });
        timeit("slab32_t256_dg", [&] { slab<32, 256, 0><<<NG(32), 256>>>(slots, dst, n, 0); });
        timeit("slab32_t256_run", [&] { slab<32, 256, 1><<<NG(32), 256>>>(slots, dst, n, 0); });
        timeit("slab24_t256_dg", [&] { slab<24, 256, 0><<<NG(24), 256>>>(slots, dst, n, 0); });
        timeit("slab24_t256_run", [&] { slab<24, 256, 1><<<NG(24), 256>>>(slots, dst, n, 0); });
        timeit("slab16_t256_run", [&] { slab<16, 256, 1><<<NG(16), 256>>>(slots, dst, n, 0); });
        timeit("slab49_t256_run_sleep7", [&] { slab<49, 256, 5><<<NG(49), 256>>>(slots, dst, n, 700); });
        timeit("slab49_t512_run_sleep7", [&] { slab<49, 512, 5><<<NG(49), 512>>>(slots, dst, n, 700); });
        timeit("slab32_t256_run_sleep7", [&] { slab<32, 256, 5><<<NG(32), 256>>>(slots, dst, n, 700); });
        timeit("slab24_t256_run_sleep7", [&] { slab<24, 256, 5><<<NG(24), 256>>>(slots, dst, n, 700); });
        timeit("slab24_t256_run_sleep3", [&] { slab<24, 256, 5><<<NG(24), 256>>>(slots, dst, n, 300); });
        printf("}");
    }
    printf("}\n");
    return 0;
}
