// ubench_rev.hip -- the config-3 shape: a seg-like kernel W (read a source buffer with
// streaming loads, write a "datagram" buffer of the same size with plain stores, 16 KiB per
// workgroup, workgroup b on XCD b mod 8) followed by a reassembly-like kernel R (copy the
// datagram buffer to a destination with non-temporal stores).  R walks the chunks forward
// or from the end, on the XCD that wrote each chunk or on another one, with plain or
// streaming loads.  When the buffer is larger than the Infinity Cache, the chunks W wrote
// last are the ones still cached: does reading them first pay, and does the reading XCD
// matter?
// Usage: ubench_rev [MiB] [iters]   -> one JSON line (µs of R = (W+R) - W)
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

constexpr uint32_t kChunk = 16384;

__global__ __launch_bounds__(256) void wk(const uint8_t *src, uint8_t *mid)
{
    const uint64_t base = (uint64_t)blockIdx.x * kChunk;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = __builtin_nontemporal_load((const G u32x4 *)(src + base + (u * 256 + threadIdx.x) * 16));
#pragma unroll
    for (int u = 0; u < 4; u++) *(G u32x4 *)(mid + base + (u * 256 + threadIdx.x) * 16) = v[u] + 1u;
}

// mode bits: 1 = reverse (XCD class kept: workgroup 8k + x takes chunk 8(K-1-k) + x),
// 2 = other XCD (chunk index + 1), 4 = nt loads
template <bool NTL>
__global__ __launch_bounds__(256) void rk(const uint8_t *mid, uint8_t *dst, uint32_t n, uint32_t mode)
{
    uint32_t c = blockIdx.x;
    if (mode & 1u) {
        const uint32_t K = n / 8, k = c / 8, x = c % 8;
        c = 8 * (K - 1 - k) + x;
    }
    if (mode & 2u) c = (c + 1) % n;
    const uint64_t base = (uint64_t)c * kChunk;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const G u32x4 *p = (const G u32x4 *)(mid + base + (u * 256 + threadIdx.x) * 16);
        v[u] = NTL ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) __builtin_nontemporal_store(v[u], (G u32x4 *)(dst + base + (u * 256 + threadIdx.x) * 16));
}

int main(int argc, char **argv)
{
    const uint64_t mib = argc > 1 ? atoll(argv[1]) : 560;
    const int iters = argc > 2 ? atoi(argv[2]) : 10;
    const uint32_t n = (uint32_t)((mib << 20) / kChunk) / 8 * 8;
    const uint64_t bytes = (uint64_t)n * kChunk;
    uint8_t *src, *mid, *dst;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&mid, bytes));
    CHECK(hipMalloc(&dst, bytes));
    CHECK(hipMemset(src, 0x5a, bytes));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto timeit = [&](int mode) {
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int i = 0; i < iters; i++) {
            wk<<<n, 256>>>(src, mid);
            if (mode < 0) continue;
            if (mode & 4) rk<true><<<n, 256>>>(mid, dst, n, (uint32_t)mode);
            else rk<false><<<n, 256>>>(mid, dst, n, (uint32_t)mode);
        }
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        return ms * 1000.0f / iters;
    };
    timeit(0);
    const float w = timeit(-1);
    printf("{\"MiB\": %llu, \"us_W\": %.2f", (unsigned long long)(bytes >> 20), w);
    const char *nm[] = {"fwd", "rev", "fwd_otherxcd", "rev_otherxcd", "fwd_nt", "rev_nt", "fwd_otherxcd_nt", "rev_otherxcd_nt"};
    for (int m = 0; m < 8; m++) {
        const float t1 = timeit(m), t2 = timeit(m);
        printf(", \"us_R_%s\": [%.2f, %.2f]", nm[m], t1 - w, t2 - w);
    }
    printf("}\n");
    return 0;
}
