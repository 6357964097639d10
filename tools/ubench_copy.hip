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
#include <cstring>
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

// Datagram-pattern copies (no header work): packets of 1472 B (36 + 1436 payload).
// MODE 10 "reas pattern": source-aligned 16-B loads of each packet slot, payload stored
//   to event + k*1436 (dword-aligned 16-B stores, edge dwords stored singly) -- the store
//   shape of reas_kernel.  MODE 11 "reas dst-aligned": destination-aligned chunks, the
//   source read at a dword-aligned offset (edge dwords singly).
template <int MODE>
__global__ __launch_bounds__(256) void patk(const uint8_t *__restrict__ pk, uint8_t *__restrict__ ev, uint32_t npk)
{
    constexpr uint32_t S = 1472, H = 36, L = 1436, SPC = 92;
    const uint32_t base = blockIdx.x * 1024 + threadIdx.x;
    u32x4 x[4];
    uint32_t ii[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t i = base + u * 256;
        ii[u] = i;
        const uint32_t p = i / SPC, c = i % SPC;
        if (p >= npk) { x[u] = u32x4{0, 0, 0, 0}; continue; }
        if (MODE == 10) {
            x[u] = *(const G u32x4 *)(pk + (uint64_t)p * S + 16 * c);
        } else {
            const uint64_t d0 = (uint64_t)p * L;                 // dst offset of payload start
            const uint64_t cb = (d0 & ~15ull) + 16ull * c;       // dst chunk
            const int64_t so = (int64_t)cb - (int64_t)d0 + H;    // src offset within packet
            const int64_t sc = so < 0 ? 0 : (so + 16 > S ? S - 16 : so);
            x[u] = *(const G u32x4_a4 *)(pk + (uint64_t)p * S + sc);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t i = ii[u];
        const uint32_t p = i / SPC, c = i % SPC;
        if (p >= npk) continue;
        if (MODE == 10) {
            const int32_t q0 = 16 * (int32_t)c;
            uint8_t *dst = ev + (int64_t)p * L + q0 - H;
            if (q0 >= (int32_t)H && q0 + 16 <= (int32_t)(H + L)) {
                __builtin_nontemporal_store(x[u], (G u32x4_a4 *)dst);
            } else {
                for (int d = 0; d < 4; d++) {
                    const int32_t q = q0 + 4 * d;
                    if (q >= (int32_t)H && q + 4 <= (int32_t)(H + L)) *(G uint32_t *)(dst + 4 * d) = x[u][d];
                }
            }
        } else {
            const uint64_t d0 = (uint64_t)p * L, d1 = d0 + L;
            const uint64_t cb = (d0 & ~15ull) + 16ull * c;
            if (cb >= d1) continue;
            if (cb >= d0 && cb + 16 <= d1) {
                __builtin_nontemporal_store(x[u], (G u32x4 *)(ev + cb));
            } else {
                for (int d = 0; d < 4; d++) {
                    const uint64_t a = cb + 4 * d;
                    if (a >= d0 && a + 4 <= d1) *(G uint32_t *)(ev + a) = x[u][d];
                }
            }
        }
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

template <int MODE>
float runpat(const uint8_t *pk, uint8_t *ev, uint32_t npk, int iters)
{
    const uint32_t grid = (npk * 92 + 1023) / 1024;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    patk<MODE><<<grid, 256>>>(pk, ev, npk);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; i++) patk<MODE><<<grid, 256>>>(pk, ev, npk);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return (float)((double)npk * (1436 + 1472) * iters / (ms * 1e-3) / 1e9);
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
    // source bytes: "one" (0x01, the default), "zero", or "random" (splitmix64 per word):
    // HBM moves mostly-zero data measurably faster than uniform random bytes
    const char *fill = argc > 3 ? argv[3] : "one";
    if (!strcmp(fill, "random")) {
        fill_random<<<(unsigned)((bytes + 64) / 8 / 256 + 1), 256>>>((uint64_t *)src, (bytes + 64) / 8);
        CHECK(hipDeviceSynchronize());
    } else {
        CHECK(hipMemset(src, strcmp(fill, "zero") ? 1 : 0, bytes + 64));
    }
    CHECK(hipMemset(dst, 0, bytes + 64));
    printf("{\"bytes\": %llu, \"iters\": %d, \"fill\": \"%s\"", (unsigned long long)bytes, iters, fill);
    printf(", \"aligned\": %.1f", run<0>(src, dst, bytes, 0, iters));
    printf(", \"aligned_nt\": %.1f", run<4>(src, dst, bytes, 0, iters));
    printf(", \"ld_mis4\": %.1f", run<1>(src, dst, bytes, 4, iters));
    printf(", \"ld_mis12\": %.1f", run<1>(src, dst, bytes, 12, iters));
    printf(", \"st_mis4\": %.1f", run<2>(src, dst, bytes, 4, iters));
    printf(", \"ld_pair_shift4\": %.1f", run<3, 4>(src, dst, bytes, 4, iters));
    printf(", \"ld_pair_shift5\": %.1f", run<3, 5>(src, dst, bytes, 5, iters));
    printf(", \"aligned_again\": %.1f", run<0>(src, dst, bytes, 0, iters));
    const uint32_t npk = (uint32_t)(bytes / 1472);
    printf(", \"pattern_reas_srcaligned\": %.1f", runpat<10>(src, dst, npk, iters));
    printf(", \"pattern_reas_dstaligned\": %.1f", runpat<11>(src, dst, npk, iters));
    printf("}\n");
    return 0;
}
