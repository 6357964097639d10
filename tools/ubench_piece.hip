// ubench_piece.hip -- does the size of a workgroup's contiguous piece change the rate of a
// copy whose source the previous kernel just wrote (the reassembly's situation)?  Kernel W
// writes `mid` from `src` (8-KiB pieces, as seg_kernel does); kernel R copies mid -> dst with
// non-temporal stores, each workgroup taking
//   contig:  one contiguous piece of R rounds x 16 KiB (round r at piece + r x 16 KiB), or
//   strided: the same number of 16-KiB blocks, round r at block r x nWG + wg, so the blocks
//            in flight at any moment are adjacent across workgroups.
// Only R is timed (events around it).  Usage: ubench_piece [MiB] [iters] -> one JSON line (µs)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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
__device__ __forceinline__ void stnt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (GA u32x4 *)p); }

__global__ __launch_bounds__(256) void wk(const uint8_t *src, uint8_t *mid)
{
    const uint64_t base = (uint64_t)blockIdx.x * 8192;
    u32x4 v[2];
#pragma unroll
    for (int u = 0; u < 2; u++) v[u] = ldnt(src + base + (u * 256 + threadIdx.x) * 16);
#pragma unroll
    for (int u = 0; u < 2; u++) *(GA u32x4 *)(mid + base + (u * 256 + threadIdx.x) * 16) = v[u] + 1u;
}

// one 16-KiB block: 256 threads x 4 chunks
__device__ __forceinline__ void block16k(const uint8_t *s, uint8_t *d)
{
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = *(const GA u32x4 *)(s + (u * 256 + threadIdx.x) * 16);
#pragma unroll
    for (int u = 0; u < 4; u++) stnt(d + (u * 256 + threadIdx.x) * 16, v[u]);
}

__global__ __launch_bounds__(256) void rk_contig(const uint8_t *mid, uint8_t *dst, int rounds)
{
    const uint64_t base = (uint64_t)blockIdx.x * rounds * 16384;
    for (int r = 0; r < rounds; r++) block16k(mid + base + (uint64_t)r * 16384, dst + base + (uint64_t)r * 16384);
}

__global__ __launch_bounds__(256) void rk_strided(const uint8_t *mid, uint8_t *dst, int rounds)
{
    for (int r = 0; r < rounds; r++) {
        const uint64_t b = ((uint64_t)r * gridDim.x + blockIdx.x) * 16384;
        block16k(mid + b, dst + b);
    }
}

int main(int argc, char **argv)
{
    const uint64_t mib = argc > 1 ? atoll(argv[1]) : 210;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    const uint64_t unit = 16384ull * 64;              // divisible by every rounds value below
    const uint64_t bytes = (mib << 20) / unit * unit;
    uint8_t *src, *mid, *dst;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&mid, bytes));
    CHECK(hipMalloc(&dst, bytes));
    CHECK(hipMemset(src, 0x5a, bytes));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto timeit = [&](int strided, int rounds) {
        const unsigned nwg = (unsigned)(bytes / (16384ull * rounds));
        float tot = 0;
        for (int i = 0; i < iters; i++) {
            wk<<<bytes / 8192, 256>>>(src, mid);
            CHECK(hipEventRecord(a));
            if (strided) rk_strided<<<nwg, 256>>>(mid, dst, rounds);
            else rk_contig<<<nwg, 256>>>(mid, dst, rounds);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            tot += ms;
        }
        CHECK(hipGetLastError());
        return tot * 1000.0f / iters;
    };
    timeit(0, 1);
    printf("{\"MiB\": %llu", (unsigned long long)(bytes >> 20));
    const int rs[] = {1, 2, 4, 8, 16};
    for (int s = 0; s < 2; s++)
        for (int r : rs) {
            const float t1 = timeit(s, r), t2 = timeit(s, r);
            printf(", \"us_%s_r%d\": [%.2f, %.2f]", s ? "strided" : "contig", r, t1, t2);
        }
    printf("}\n");
    return 0;
}
