// ubench_store.hip -- plain 16-B copies on gfx950 by load and store cache policy.
//
// For the copy calibration the bench reports beside its roofline and for the store policy
// of the SAR kernels' outputs: GB/s (read + write bytes / time) of a copy of N MiB of
// uniform random bytes, one 16-KiB piece per 256-thread workgroup (four 16-B loads per
// thread issued before the stores), launched back to back.
//   loads : plain | nt
//   stores: plain | nt | sc1 (write-through: the line leaves the XCD's L2) | sc1 nt
// Usage: ubench_store [MiB] [iters]   -> one JSON line
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

template <int LD, int ST, int U>
__global__ __launch_bounds__(256) void copyk(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, uint64_t nch)
{
    const uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t i = base + (uint64_t)u * 256;
        const uint64_t j = i < nch ? i : 0;
        if (LD == 1) v[u] = __builtin_nontemporal_load((const G u32x4 *)(src + 16 * j));
        else v[u] = *(const G u32x4 *)(src + 16 * j);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t i = base + (uint64_t)u * 256;
        if (i >= nch) continue;
        uint8_t *p = dst + 16 * i;
        if (ST == 0) *(G u32x4 *)p = v[u];
        else if (ST == 1) __builtin_nontemporal_store(v[u], (G u32x4 *)p);
        else if (ST == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v[u]) : "memory");
        else asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" ::"v"(p), "v"(v[u]) : "memory");
    }
}

__global__ void fill_random(uint64_t *p, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
}

template <int LD, int ST, int U>
float run(const uint8_t *src, uint8_t *dst, uint64_t bytes, int iters)
{
    const uint64_t nch = bytes / 16;
    const uint32_t grid = (uint32_t)((nch + 256 * U - 1) / (256 * U));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    copyk<LD, ST, U><<<grid, 256>>>(src, dst, nch);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; i++) copyk<LD, ST, U><<<grid, 256>>>(src, dst, nch);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return (float)(2.0 * 16 * nch * iters / (ms * 1e-3) / 1e9);
}

int main(int argc, char **argv)
{
    const uint64_t mib = argc > 1 ? atoll(argv[1]) : 1024;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    const uint64_t bytes = mib << 20;
    uint8_t *src, *dst;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&dst, bytes));
    fill_random<<<(unsigned)(bytes / 8 / 256 + 1), 256>>>((uint64_t *)src, bytes / 8);
    CHECK(hipMemset(dst, 0, bytes));
    CHECK(hipDeviceSynchronize());
    printf("{\"MiB\": %llu, \"iters\": %d, \"data\": \"random\"", (unsigned long long)mib, iters);
    printf(", \"ld_plain_st_plain\": %.1f", run<0, 0, 4>(src, dst, bytes, iters));
    printf(", \"ld_nt_st_plain\": %.1f", run<1, 0, 4>(src, dst, bytes, iters));
    printf(", \"ld_plain_st_nt\": %.1f", run<0, 1, 4>(src, dst, bytes, iters));
    printf(", \"ld_nt_st_nt\": %.1f", run<1, 1, 4>(src, dst, bytes, iters));
    printf(", \"ld_nt_st_sc1\": %.1f", run<1, 2, 4>(src, dst, bytes, iters));
    printf(", \"ld_nt_st_sc1nt\": %.1f", run<1, 3, 4>(src, dst, bytes, iters));
    printf(", \"ld_plain_st_sc1\": %.1f", run<0, 2, 4>(src, dst, bytes, iters));
    printf(", \"ld_nt_st_nt_U8\": %.1f", run<1, 1, 8>(src, dst, bytes, iters));
    printf(", \"ld_nt_st_sc1_U8\": %.1f", run<1, 2, 8>(src, dst, bytes, iters));
    printf(", \"ld_nt_st_nt_U2\": %.1f", run<1, 1, 2>(src, dst, bytes, iters));
    printf(", \"ld_nt_st_nt_again\": %.1f", run<1, 1, 4>(src, dst, bytes, iters));
    printf("}\n");
    return 0;
}
