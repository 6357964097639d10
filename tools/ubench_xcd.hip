// ubench_xcd.hip -- does work placement across the 8 XCDs limit a streaming copy?
//
// Copies `MiB` of 16-byte-aligned data three ways and prints GB/s (read + write bytes):
//   static : one workgroup per 16 KiB of output (the hardware dispatcher hands
//            workgroups to XCDs round-robin, so every XCD moves 1/8 of the bytes)
//   dyn1   : a resident grid (8 workgroups per CU) pulling 64 KiB units from ONE
//            atomic counter, so a faster XCD takes more units
//   dyn8   : the same with one counter per XCD (range = 1/8 of the units each) and
//            stealing from the other XCDs' ranges when the own range is empty
// plus, for static, the median workgroup duration per XCD (s_memrealtime).
// Usage: ubench_xcd [MiB] [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

__device__ __forceinline__ uint32_t xcc_id()
{
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 0xF;
}

// 256 threads x 4 chunks of 16 B = 16 KiB per round
__device__ __forceinline__ void copy_round(const uint8_t *src, uint8_t *dst, uint64_t c0, uint64_t nch)
{
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint64_t i = c0 + (uint64_t)u * 256 + threadIdx.x;
        if (i < nch) v[u] = __builtin_nontemporal_load((const G u32x4 *)(src + 16 * i));
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint64_t i = c0 + (uint64_t)u * 256 + threadIdx.x;
        if (i < nch) __builtin_nontemporal_store(v[u], (G u32x4 *)(dst + 16 * i));
    }
}

__global__ __launch_bounds__(256) void copy_static(const uint8_t *src, uint8_t *dst, uint64_t nch, uint64_t *trace)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    copy_round(src, dst, (uint64_t)blockIdx.x * 1024, nch);
    if (trace) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            trace[2 * blockIdx.x] = ((uint64_t)xcc_id() << 60) | t0;
            trace[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

// default-policy (or nt) copy with per-workgroup XCD timing: read what the previous kernel wrote
template <bool NTLD, bool NTST>
__global__ __launch_bounds__(256) void copy_static_pol(const uint8_t *src, uint8_t *dst, uint64_t nch, uint64_t *trace)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t c0 = (uint64_t)blockIdx.x * 1024;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint64_t i = c0 + (uint64_t)u * 256 + threadIdx.x;
        if (i < nch) v[u] = NTLD ? __builtin_nontemporal_load((const G u32x4 *)(src + 16 * i)) : *(const G u32x4 *)(src + 16 * i);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint64_t i = c0 + (uint64_t)u * 256 + threadIdx.x;
        if (i < nch) {
            if (NTST) __builtin_nontemporal_store(v[u], (G u32x4 *)(dst + 16 * i));
            else *(G u32x4 *)(dst + 16 * i) = v[u];
        }
    }
    if (trace) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            trace[2 * blockIdx.x] = ((uint64_t)xcc_id() << 60) | t0;
            trace[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

constexpr uint32_t kUnitRounds = 4;   // 64 KiB per unit

__global__ __launch_bounds__(256) void copy_dyn1(const uint8_t *src, uint8_t *dst, uint64_t nch, uint32_t nUnits,
                                                 uint32_t *ctr)
{
    __shared__ uint32_t sU;
    for (;;) {
        if (threadIdx.x == 0) sU = atomicAdd(ctr, 1u);
        __syncthreads();
        const uint32_t u = sU;
        __syncthreads();
        if (u >= nUnits) break;
        for (uint32_t r = 0; r < kUnitRounds; r++)
            copy_round(src, dst, ((uint64_t)u * kUnitRounds + r) * 1024, nch);
    }
}

__global__ __launch_bounds__(256) void copy_dyn8(const uint8_t *src, uint8_t *dst, uint64_t nch, uint32_t nUnits,
                                                 uint32_t *ctr /* 8 counters, 64 B apart */)
{
    __shared__ uint32_t sU;
    const uint32_t x = xcc_id() & 7u;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t got = 0xFFFFFFFFu;
            for (uint32_t k = 0; k < 8 && got == 0xFFFFFFFFu; k++) {
                const uint32_t q = (x + k) & 7u;
                const uint32_t lo = (uint32_t)((uint64_t)q * nUnits / 8), hi = (uint32_t)((uint64_t)(q + 1) * nUnits / 8);
                if (__hip_atomic_load(ctr + 16 * q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= hi - lo) continue;
                const uint32_t v = atomicAdd(ctr + 16 * q, 1u);
                if (v < hi - lo) got = lo + v;
            }
            sU = got;
        }
        __syncthreads();
        const uint32_t u = sU;
        __syncthreads();
        if (u == 0xFFFFFFFFu) break;
        for (uint32_t r = 0; r < kUnitRounds; r++)
            copy_round(src, dst, ((uint64_t)u * kUnitRounds + r) * 1024, nch);
    }
}

int main(int argc, char **argv)
{
    const uint64_t mib = argc > 1 ? atoll(argv[1]) : 256;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    const uint64_t bytes = mib << 20, nch = bytes / 16;
    uint8_t *src, *dst;
    uint32_t *ctr;
    uint64_t *trace;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&dst, bytes));
    CHECK(hipMalloc(&ctr, 8 * 64));
    const uint32_t nStatic = (uint32_t)((nch + 1023) / 1024);
    CHECK(hipMalloc(&trace, (size_t)nStatic * 16));
    CHECK(hipMemset(src, 1, bytes));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t nUnits = (uint32_t)((nch + 1024 * kUnitRounds - 1) / (1024 * kUnitRounds));
    const uint32_t grid = (uint32_t)cus * 8;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timeit = [&](int which) {
        float best = 1e30f, sum = 0;
        for (int i = 0; i < iters + 2; i++) {
            CHECK(hipMemsetAsync(ctr, 0, 8 * 64));
            CHECK(hipEventRecord(e0));
            if (which == 0) copy_static<<<nStatic, 256>>>(src, dst, nch, nullptr);
            else if (which == 1) copy_dyn1<<<grid, 256>>>(src, dst, nch, nUnits, ctr);
            else copy_dyn8<<<grid, 256>>>(src, dst, nch, nUnits, ctr);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (i >= 2) {
                sum += ms;
                best = std::min(best, ms);
            }
        }
        return 2.0 * bytes / (sum / iters * 1e-3) / 1e9;
    };
    const double gs = timeit(0), g1 = timeit(1), g8 = timeit(2);
    // static: per-XCD durations
    copy_static<<<nStatic, 256>>>(src, dst, nch, trace);
    CHECK(hipDeviceSynchronize());
    std::vector<uint64_t> t((size_t)nStatic * 2);
    CHECK(hipMemcpy(t.data(), trace, t.size() * 8, hipMemcpyDeviceToHost));
    std::vector<std::vector<double>> d(16);
    for (uint32_t b = 0; b < nStatic; b++) {
        const uint32_t x = (uint32_t)(t[2 * b] >> 60);
        const uint64_t s = t[2 * b] & ((1ull << 60) - 1);
        d[x & 15].push_back((double)(t[2 * b + 1] - s) * 0.01);
    }
    printf("{\"MiB\": %llu, \"static_GBps\": %.1f, \"dyn1_GBps\": %.1f, \"dyn8_GBps\": %.1f, \"static_block_us_median_by_xcc\": [",
           (unsigned long long)mib, gs, g1, g8);
    for (int x = 0; x < 8; x++) {
        auto &v = d[x];
        std::sort(v.begin(), v.end());
        printf("%s%.2f", x ? ", " : "", v.empty() ? 0.0 : v[v.size() / 2]);
    }
    printf("]");
    // chain: A -> B (default stores), then B -> C timed per XCD: fresh data in the
    // Infinity Cache, as when reas_kernel reads what seg_kernel just wrote
    uint8_t *C;
    CHECK(hipMalloc(&C, bytes));
    auto per_xcc = [&](const char *name) {
        CHECK(hipMemcpy(t.data(), trace, t.size() * 8, hipMemcpyDeviceToHost));
        std::vector<std::vector<double>> dd(16);
        uint64_t tmin = ~0ull, tmax = 0;
        for (uint32_t b = 0; b < nStatic; b++) {
            const uint64_t s0 = t[2 * b] & ((1ull << 60) - 1);
            dd[(t[2 * b] >> 60) & 15].push_back((double)(t[2 * b + 1] - s0) * 0.01);
            tmin = std::min(tmin, s0);
            tmax = std::max(tmax, t[2 * b + 1]);
        }
        printf(", \"%s_span_us\": %.1f, \"%s_by_xcc\": [", name, (tmax - tmin) * 0.01, name);
        for (int x = 0; x < 8; x++) {
            auto &v = dd[x];
            std::sort(v.begin(), v.end());
            printf("%s%.2f", x ? ", " : "", v.empty() ? 0.0 : v[v.size() / 2]);
        }
        printf("]");
    };
    for (int rep = 0; rep < 3; rep++) {
        copy_static_pol<true, false><<<nStatic, 256>>>(src, dst, nch, nullptr);
        copy_static_pol<false, true><<<nStatic, 256>>>(dst, C, nch, trace);
    }
    CHECK(hipDeviceSynchronize());
    per_xcc("fresh_read");
    for (int rep = 0; rep < 3; rep++) {
        copy_static_pol<true, true><<<nStatic, 256>>>(src, dst, nch, nullptr);
        copy_static_pol<false, true><<<nStatic, 256>>>(dst, C, nch, trace);
    }
    CHECK(hipDeviceSynchronize());
    per_xcc("after_nt_write");
    printf("}\n");
    return 0;
}
