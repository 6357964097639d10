// ubench_copy.hip -- calibration microbenchmark for the SAR copy kernels on gfx950.
//
// Measures HBM copy rate (GB/s, read+write bytes / time) for the access shapes the
// segment/reassemble kernels can use:
//   aligned      : 16-B aligned loads and stores (the "achievable HBM" calibration)
//   ld_mis4      : source offset by 4 B (dword-aligned dwordx4 loads), aligned stores
//   st_mis4      : aligned loads, destination offset by 4 B
//   ld_pair      : aligned loads of two neighbouring chunks + v_alignbyte funnel shift
//   aligned_nt   : aligned copy with non-temporal loads/stores
// Usage: ubench_copy [MiB] [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(4))) u32x4_a4;
#define G __attribute__((address_space(1)))

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

template <int MODE, int U, int SH = 0>
__global__ __launch_bounds__(256) void copyk(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                              uint64_t nchunks, uint32_t shiftBytes)
{
    const uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t i = base + (uint64_t)u * 256;
        if (i >= nchunks) continue;
        if (MODE == 0 || MODE == 2) {
            v[u] = *(const G u32x4 *)(src + 16 * i);
        } else if (MODE == 1) {
            v[u] = *(const G u32x4_a4 *)(src + 16 * i + shiftBytes);
        } else if (MODE == 3) {
            const u32x4 a = *(const G u32x4 *)(src + 16 * i);
            const u32x4 b = *(const G u32x4 *)(src + 16 * i + 16);
            constexpr int q = SH >> 2, r = SH & 3;
            const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            u32x4 o;
            // funnel shift by q dwords + r bytes
            o.x = __builtin_amdgcn_alignbyte(w[(q + 1) & 7], w[q & 7], r);
            o.y = __builtin_amdgcn_alignbyte(w[(q + 2) & 7], w[(q + 1) & 7], r);
            o.z = __builtin_amdgcn_alignbyte(w[(q + 3) & 7], w[(q + 2) & 7], r);
            o.w = __builtin_amdgcn_alignbyte(w[(q + 4) & 7], w[(q + 3) & 7], r);
            v[u] = o;
        } else if (MODE == 4) {
            v[u] = __builtin_nontemporal_load((const G u32x4 *)(src + 16 * i));
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t i = base + (uint64_t)u * 256;
        if (i >= nchunks) continue;
        if (MODE == 2)
            *(G u32x4_a4 *)(dst + 16 * i + shiftBytes) = v[u];
        else if (MODE == 4)
            __builtin_nontemporal_store(v[u], (G u32x4 *)(dst + 16 * i));
        else
            *(G u32x4 *)(dst + 16 * i) = v[u];
    }
}

template <int MODE, int SH = 0>
float run(const uint8_t *src, uint8_t *dst, uint64_t bytes, uint32_t shift, int iters)
{
    constexpr int U = 4;
    const uint64_t nch = bytes / 16 - 2;
    const uint32_t grid = (uint32_t)((nch + 256 * U - 1) / (256 * U));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    copyk<MODE, U, SH><<<grid, 256>>>(src, dst, nch, shift);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; i++) copyk<MODE, U, SH><<<grid, 256>>>(src, dst, nch, shift);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return (float)(2.0 * 16 * nch * iters / (ms * 1e-3) / 1e9);
}

int main(int argc, char **argv)
{
    const uint64_t mib = argc > 1 ? atoll(argv[1]) : 1024;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    const uint64_t bytes = mib << 20;
    uint8_t *src, *dst;
    CHECK(hipMalloc(&src, bytes + 64));
    CHECK(hipMalloc(&dst, bytes + 64));
    CHECK(hipMemset(src, 1, bytes + 64));
    printf("{\"bytes\": %llu, \"iters\": %d", (unsigned long long)bytes, iters);
    printf(", \"aligned\": %.1f", run<0>(src, dst, bytes, 0, iters));
    printf(", \"aligned_nt\": %.1f", run<4>(src, dst, bytes, 0, iters));
    printf(", \"ld_mis4\": %.1f", run<1>(src, dst, bytes, 4, iters));
    printf(", \"ld_mis12\": %.1f", run<1>(src, dst, bytes, 12, iters));
    printf(", \"st_mis4\": %.1f", run<2>(src, dst, bytes, 4, iters));
    printf(", \"ld_pair_shift4\": %.1f", run<3, 4>(src, dst, bytes, 4, iters));
    printf(", \"ld_pair_shift5\": %.1f", run<3, 5>(src, dst, bytes, 5, iters));
    printf(", \"aligned_again\": %.1f", run<0>(src, dst, bytes, 0, iters));
    printf("}\n");
    return 0;
}
