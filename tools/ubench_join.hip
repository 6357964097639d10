// ubench_join.hip -- does a datagram boundary's 16-byte destination chunk cost HBM traffic
// when two lanes write its two parts?  (reas_kernel's PMC: writes 1.043x, reads 1.022x the
// algorithmic bytes, ~62 B per datagram; VERDICT r4 "attack the write side first".)
//
// Copy-only kernels over the headline batch's datagram slots (1472-B slots, 36-B headers,
// 1436-B payloads, one contiguous event per 731 datagrams), destination-aligned as
// reas_kernel (chunk c of datagram p covers event bytes [(p*1436 & ~15) + 16c, +16)):
//   split<G> : both partial chunks of a boundary written by their own datagram's lane
//              (dword / dwordx2 / dwordx3 edge stores): today's reas_kernel
//   join<G>  : the lane of p's last chunk also loads p+1's first window and writes the whole
//              16 bytes; p+1's chunk-0 lane stores nothing
//   lin<G>   : destination-space lanes: lane j writes event chunk j of the group's range,
//              loading one or two windows (every store whole except the group's two edges)
// G datagrams per 256-thread workgroup, one 1024-chunk round per workgroup at G = 8, rounds
// of 1024 chunks otherwise.  Usage: ubench_join [iters] -> one JSON line (median us).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GA __attribute__((address_space(1)))
typedef u32x4 __attribute__((aligned(4))) u32x4_a4;

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

constexpr uint32_t kStride = 1472, kHl = 36, kPl = 1436, kSpc = kStride / 16, kPerEv = 731;

__device__ __forceinline__ u32x4 ld(const uint8_t *p) { return *(const GA u32x4_a4 *)p; }
__device__ __forceinline__ void stnt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (GA u32x4 *)p); }
__device__ __forceinline__ u32x4 rot(u32x4 x, uint32_t s)
{
    return s == 0 ? x : s == 1 ? u32x4{x.y, x.z, x.w, 0u} : s == 2 ? u32x4{x.z, x.w, 0u, 0u} : u32x4{x.w, 0u, 0u, 0u};
}
// event offset of datagram P's payload (events of 731 datagrams, 1 MiB each)
__device__ __forceinline__ uint64_t pofs(uint32_t P)
{
    return (uint64_t)(P / kPerEv) * 1048576ull + (uint64_t)(P % kPerEv) * kPl;
}
__device__ __forceinline__ uint32_t plen(uint32_t P) { return (P % kPerEv == kPerEv - 1) ? 1048576u - 730u * kPl : kPl; }
// window of chunk c of a payload of phase a inside its slot: start and slide
__device__ __forceinline__ uint32_t win(uint32_t c, uint32_t a, uint32_t &sh)
{
    uint32_t r = kHl + 16u * c - a;
    sh = (r + 16u > kStride) ? (r + 16u - kStride) >> 2 : 0u;
    return r - 4u * sh;
}
__device__ __forceinline__ void st_edge(uint8_t *D, u32x4 o, uint32_t lo, uint32_t hi)
{
    for (uint32_t w = lo / 4; w < hi / 4; w++) *(GA uint32_t *)(D + 4 * w) = o[w];
}

template <int G, int MODE>   // MODE 0 split, 1 join
__global__ __launch_bounds__(256) void dgk(const uint8_t *slots, uint8_t *dst, uint32_t n)
{
    const uint32_t pg = blockIdx.x * G;
    const uint32_t gn = (n - pg < G) ? n - pg : G;
    const uint32_t nch = gn * kSpc;
    for (uint32_t r0 = 0; r0 < nch; r0 += 1024) {
        u32x4 x[4], y[4];
        uint32_t pp[4], cc[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = r0 + u * 256 + threadIdx.x;
            const uint32_t ic = i < nch ? i : 0u;
            const uint32_t p = ic / kSpc, c = ic - p * kSpc, P = pg + p;
            pp[u] = i < nch ? p : 0xFFFFFFFFu;
            cc[u] = c;
            const uint32_t a = (uint32_t)pofs(P) & 15u, L = plen(P);
            uint32_t sh, off = 0;
            if (i < nch && 16u * c < a + L) off = P * kStride + win(c, a, sh);
            x[u] = ld(slots + off);
            y[u] = u32x4{0, 0, 0, 0};
            if (MODE == 1) {
                const uint32_t e = a + L;
                if (i < nch && c == (e - 1u) / 16u && (e & 15u) && p + 1u < gn && P % kPerEv != kPerEv - 1)
                    y[u] = ld(slots + (uint64_t)(P + 1u) * kStride + kHl - (e & 15u));
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (pp[u] == 0xFFFFFFFFu) continue;
            const uint32_t p = pp[u], c = cc[u], P = pg + p;
            const uint64_t ofs = pofs(P);
            const uint32_t a = (uint32_t)ofs & 15u, L = plen(P), e = a + L;
            if (16u * c >= e) continue;
            uint8_t *D = dst + (ofs & ~15ull) + 16ull * c;
            uint32_t sh;
            (void)win(c, a, sh);
            const u32x4 o = rot(x[u], sh);
            const uint32_t lo = c == 0 ? a : 0u, hi = (e - 16u * c < 16u) ? e - 16u * c : 16u;
            if (MODE == 1) {
                if (c == 0 && a != 0 && p > 0 && P % kPerEv != 0) continue;          // joined by p-1
                if (hi < 16u && p + 1u < gn && P % kPerEv != kPerEv - 1) {
                    const uint32_t k = hi >> 2;
                    stnt(D, u32x4{o.x, k > 1 ? o.y : y[u].y, k > 2 ? o.z : y[u].z, y[u].w});
                    continue;
                }
            }
            if (lo == 0 && hi == 16) stnt(D, o);
            else st_edge(D, o, lo, hi);
        }
    }
}

// destination-space: the group's datagrams [pg, pg+gn) cover event bytes [b0, b1) (within
// one event here only when the group does not cross an event; groups that do are split at
// the event edge by processing chunk ranges per event)
template <int G>
__global__ __launch_bounds__(256) void lin(const uint8_t *slots, uint8_t *dst, uint32_t n)
{
    const uint32_t pg = blockIdx.x * G;
    const uint32_t gn = (n - pg < G) ? n - pg : G;
    const uint64_t b0 = pofs(pg), b1 = pofs(pg + gn - 1) + plen(pg + gn - 1);
    const uint64_t c0 = b0 >> 4, c1 = (b1 + 15) >> 4;
    for (uint64_t j0 = c0; j0 < c1; j0 += 1024) {
        u32x4 x[4], y[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t j = j0 + u * 256 + threadIdx.x;
            x[u] = y[u] = u32x4{0, 0, 0, 0};
            if (j >= c1) continue;
            const uint64_t B = 16 * j;                      // chunk start (event space)
            const uint64_t ev = B >> 20;
            const uint64_t q = (B & 1048575ull);
            uint32_t k = (uint32_t)(q / kPl);               // datagram of the chunk's first byte
            const uint32_t P = (uint32_t)ev * kPerEv + k;
            const uint32_t s = (uint32_t)(q - (uint64_t)k * kPl);   // byte within the payload (multiple of 4)
            // first window: payload bytes [s, s+16) of datagram P (slid back at the slot end)
            uint32_t r = kHl + s, sh = 0;
            if (r + 16u > kStride) { sh = (r + 16u - kStride) >> 2; r -= 4u * sh; }
            x[u] = ld(slots + (uint64_t)P * kStride + r);
            x[u] = rot(x[u], sh);
            if (s + 16u > kPl && k < kPerEv - 1) {         // spills into P + 1
                const uint32_t t = kPl - s;                 // bytes from P
                y[u] = ld(slots + (uint64_t)(P + 1) * kStride + kHl - t);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t j = j0 + u * 256 + threadIdx.x;
            if (j >= c1) continue;
            const uint64_t B = 16 * j;
            const uint32_t s = (uint32_t)((B & 1048575ull) % kPl);
            const uint32_t t = (s + 16u > kPl) ? (kPl - s) >> 2 : 4u;
            const u32x4 m{x[u].x, t > 1 ? x[u].y : y[u].y, t > 2 ? x[u].z : y[u].z, t > 3 ? x[u].w : y[u].w};
            const uint64_t lo = B < b0 ? b0 - B : 0, hi = B + 16 > b1 ? b1 - B : 16;
            if (lo == 0 && hi == 16) stnt(dst + B, m);
            else st_edge(dst + B, m, (uint32_t)lo, (uint32_t)hi);
        }
    }
}

__global__ __launch_bounds__(256) void fill_random(uint8_t *p, uint64_t n16, uint64_t seed)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        *(GA u32x4 *)(p + 16 * i) = u32x4{(uint32_t)z, (uint32_t)(z >> 32), (uint32_t)(z * 3), (uint32_t)(z >> 7)};
    }
}
__global__ __launch_bounds__(256) void wk_slots(const uint8_t *src, uint8_t *slots, uint64_t bytes)
{
    const uint64_t base = (uint64_t)blockIdx.x * 8192;
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const uint64_t o = base + (u * 256 + threadIdx.x) * 16;
        if (o < bytes) *(GA u32x4 *)(slots + o) = __builtin_nontemporal_load((const GA u32x4 *)(src + o));
    }
}
__global__ void cmp(const uint8_t *a, const uint8_t *b, uint64_t n, unsigned long long *bad)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (a[i] != b[i]) atomicAdd(bad, 1ull);
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 15;
    const uint32_t nev = 200, n = nev * kPerEv;        // 146,200 datagrams, 215 MB of slots
    const uint64_t sbytes = (uint64_t)n * kStride, ebytes = (uint64_t)nev << 20;
    uint8_t *src, *slots, *dst, *ref;
    CHECK(hipMalloc(&src, sbytes));
    CHECK(hipMalloc(&slots, sbytes + 4096));
    CHECK(hipMalloc(&dst, ebytes));
    CHECK(hipMalloc(&ref, ebytes));
    unsigned long long *bad;
    CHECK(hipMalloc(&bad, 8));
    fill_random<<<4096, 256>>>(src, sbytes / 16, 777);
    wk_slots<<<(unsigned)((sbytes + 8191) / 8192), 256>>>(src, slots, sbytes);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto timeit = [&](auto launch) {
        std::vector<float> v;
        for (int i = 0; i < iters; i++) {
            wk_slots<<<(unsigned)((sbytes + 8191) / 8192), 256>>>(src, slots, sbytes);
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
    auto check = [&](const char *name) {
        CHECK(hipMemset(bad, 0, 8));
        cmp<<<4096, 256>>>(dst, ref, ebytes, bad);
        unsigned long long h = 0;
        CHECK(hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost));
        if (h) fprintf(stderr, "%s: %llu bytes differ\n", name, h);
        return h == 0;
    };
#define NG(G) (unsigned)((n + (G) - 1) / (G))
    dgk<8, 0><<<NG(8), 256>>>(slots, ref, n);
    CHECK(hipDeviceSynchronize());
    printf("{\"datagrams\": %u", n);
    for (int rep = 0; rep < 2; rep++) {
        printf(", \"rep%d\": {", rep);
        printf("\"split8\": %.2f", timeit([&] { dgk<8, 0><<<NG(8), 256>>>(slots, dst, n); }));
        printf(", \"join8\": %.2f", timeit([&] { dgk<8, 1><<<NG(8), 256>>>(slots, dst, n); }));
        if (!check("join8")) return 1;
        printf(", \"lin8\": %.2f", timeit([&] { lin<8><<<NG(8), 256>>>(slots, dst, n); }));
        if (!check("lin8")) return 1;
        printf(", \"split59\": %.2f", timeit([&] { dgk<59, 0><<<NG(59), 256>>>(slots, dst, n); }));
        printf(", \"join59\": %.2f", timeit([&] { dgk<59, 1><<<NG(59), 256>>>(slots, dst, n); }));
        if (!check("join59")) return 1;
        printf(", \"lin59\": %.2f", timeit([&] { lin<59><<<NG(59), 256>>>(slots, dst, n); }));
        if (!check("lin59")) return 1;
        printf("}");
    }
    printf("}\n");
    return 0;
}
