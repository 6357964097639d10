// ubench_local.hip -- can a round trip through memory be served by the writer's L2?  The
// floor of the device-resident segment -> reassemble step without its header work: copy a
// source buffer to a "datagram" buffer and that buffer on to a destination.
//   two:   kernel W (streaming source loads, plain stores to mid), then kernel R (mid -> dst,
//          streaming stores) -- the two-launch shape of seg_kernel + reas_kernel;
//   local: ONE kernel; each workgroup copies its piece src -> mid, waits for its own stores
//          (s_waitcnt vmcnt(0) + barrier), then reads the piece back with L1-bypassing (sc1)
//          loads -- from its own XCD's L2 if the lines are still there -- and stores it to dst.
// Usage: ubench_local [MiB] [iters]   -> one JSON line (µs per pass)
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

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const G u32x4 *)p); }
__device__ __forceinline__ void stnt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (G u32x4 *)p); }
// sc1 (L1-bypassing) 16-byte load through a buffer resource whose base is workgroup-uniform
__device__ __forceinline__ u32x4 ldsc1(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16);
}

template <int U>
__global__ __launch_bounds__(256) void wk(const uint8_t *src, uint8_t *mid)
{
    const uint64_t base = (uint64_t)blockIdx.x * (256 * 16 * U);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = ldnt(src + base + (u * 256 + threadIdx.x) * 16);
#pragma unroll
    for (int u = 0; u < U; u++) *(G u32x4 *)(mid + base + (u * 256 + threadIdx.x) * 16) = v[u] + 1u;
}

template <int U>
__global__ __launch_bounds__(256) void rk(const uint8_t *mid, uint8_t *dst)
{
    const uint64_t base = (uint64_t)blockIdx.x * (256 * 16 * U);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = *(const G u32x4 *)(mid + base + (u * 256 + threadIdx.x) * 16);
#pragma unroll
    for (int u = 0; u < U; u++) stnt(dst + base + (u * 256 + threadIdx.x) * 16, v[u]);
}

// R = rounds per workgroup: the piece is R x (256 x 16 x U) bytes, written then read back
template <int U, int R>
__global__ __launch_bounds__(256) void local(const uint8_t *src, uint8_t *mid, uint8_t *dst)
{
    constexpr uint64_t RB = 256 * 16 * U;
    const uint64_t base = (uint64_t)blockIdx.x * RB * R;
    for (int r = 0; r < R; r++) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ldnt(src + base + r * RB + (u * 256 + threadIdx.x) * 16);
#pragma unroll
        for (int u = 0; u < U; u++) *(G u32x4 *)(mid + base + r * RB + (u * 256 + threadIdx.x) * 16) = v[u] + 1u;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(mid + base, (short)0, 0x7FFFFFFF, 0x00020000);
    for (int r = 0; r < R; r++) {
        u32x4 v[U];
        // read back another thread's chunk (a rotation), so nothing comes from registers
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ldsc1(rs, (uint32_t)(r * RB + (u * 256 + ((threadIdx.x + 64) & 255)) * 16));
#pragma unroll
        for (int u = 0; u < U; u++) stnt(dst + base + r * RB + (u * 256 + ((threadIdx.x + 64) & 255)) * 16, v[u]);
    }
}

int main(int argc, char **argv)
{
    const uint64_t mib = argc > 1 ? atoll(argv[1]) : 221;
    const int iters = argc > 2 ? atoi(argv[2]) : 10;
    const uint64_t bytes = (mib << 20) / 65536 * 65536;
    uint8_t *src, *mid, *dst;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&mid, bytes));
    CHECK(hipMalloc(&dst, bytes));
    CHECK(hipMemset(src, 0x5a, bytes));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto timeit = [&](int v) {
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int i = 0; i < iters; i++) {
            switch (v) {
            case 0: wk<2><<<bytes / 8192, 256>>>(src, mid); rk<4><<<bytes / 16384, 256>>>(mid, dst); break;
            case 1: wk<2><<<bytes / 8192, 256>>>(src, mid); break;
            case 2: local<2, 1><<<bytes / 8192, 256>>>(src, mid, dst); break;
            case 3: local<4, 1><<<bytes / 16384, 256>>>(src, mid, dst); break;
            case 4: local<2, 4><<<bytes / 32768, 256>>>(src, mid, dst); break;
            case 5: local<1, 1><<<bytes / 4096, 256>>>(src, mid, dst); break;
            }
        }
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        CHECK(hipGetLastError());
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        return ms * 1000.0f / iters;
    };
    timeit(0);
    const char *nm[] = {"two_launch", "W_only", "local_8k", "local_16k", "local_32k_4rounds", "local_4k"};
    printf("{\"MiB\": %llu", (unsigned long long)(bytes >> 20));
    for (int v = 0; v < 6; v++) {
        const float t1 = timeit(v), t2 = timeit(v);
        printf(", \"us_%s\": [%.2f, %.2f]", nm[v], t1, t2);
    }
    printf("}\n");
    return 0;
}
