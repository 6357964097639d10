// ubench_l2keep.hip -- do lines a kernel stores stay readable from the storing XCD's L2 by
// the NEXT kernel (same stream)?
//
// Kernel W: one workgroup per 16-KiB chunk of a buffer of `MiB`, plain (or nt) 16-byte
// stores; each workgroup records the XCD it ran on (owner[chunk]).  Kernel R: a resident
// grid in which every workgroup pulls chunks from a per-XCD list (built on the host from
// owner[]) and sums them: "match" reads the chunks its own XCD wrote, "mismatch" those
// XCD (x+1) mod 8 wrote.  Times W + R pairs with HIP events; R alone is the difference to
// W alone.  If the next kernel's acquire drops the storing XCD's L2 (or its write-back at
// the kernel boundary evicts it), match == mismatch.
// Usage: ubench_l2keep [MiB] [iters]   -> one JSON line
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

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

__device__ __forceinline__ uint32_t xcc_id()
{
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 0x7;
}

constexpr uint32_t kChunk = 16384;

template <int NT>
__global__ __launch_bounds__(256) void wk(uint8_t *buf, uint32_t *owner, uint32_t seed)
{
    uint8_t *p = buf + (uint64_t)blockIdx.x * kChunk;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t i = (u * 256 + threadIdx.x) * 16;
        const u32x4 v{seed + i, seed ^ i, i * 3u, blockIdx.x};
        if (NT) __builtin_nontemporal_store(v, (G u32x4 *)(p + i));
        else *(G u32x4 *)(p + i) = v;
    }
    if (threadIdx.x == 0) owner[blockIdx.x] = xcc_id();
}

// lists: 8 lists of chunk indices, list x at lists + x * cap, length len[x]; heads[8]
__global__ __launch_bounds__(256) void rk(const uint8_t *buf, const uint32_t *lists, const uint32_t *len,
                                          uint32_t cap, uint32_t *heads, uint32_t shift, uint32_t *sink)
{
    __shared__ uint32_t s_idx;
    const uint32_t x = (xcc_id() + shift) & 7u;
    u32x4 acc{0, 0, 0, 0};
    for (;;) {
        if (threadIdx.x == 0) s_idx = atomicAdd(heads + x, 1u);
        __syncthreads();
        const uint32_t k = s_idx;
        __syncthreads();
        if (k >= len[x]) break;
        const uint8_t *p = buf + (uint64_t)lists[x * cap + k] * kChunk;
#pragma unroll
        for (int u = 0; u < 4; u++) acc += *(const G u32x4 *)(p + (u * 256 + threadIdx.x) * 16);
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = 1u;
}

// static form: workgroup b reads chunk (b + shift) mod n -- the dispatcher's round-robin is
// the same for W and R (same grid), so shift 0 reads what the same XCD wrote, shift 8 what
// the same XCD wrote 8 workgroups later; rev: XCD-class-reversed order (workgroup 8k + x
// reads chunk 8(K-1-k) + x: same XCD, most recently written first); copy: also store the
// chunk to dst (nt), the shape of a reassembly read + event write
template <bool COPY>
__global__ __launch_bounds__(256) void rs(const uint8_t *buf, uint8_t *dst, uint32_t n, uint32_t shift, int rev,
                                          uint32_t *sink)
{
    uint32_t c = (blockIdx.x + shift) % n;
    if (rev) {
        const uint32_t K = n / 8, k = blockIdx.x / 8, x = blockIdx.x % 8;
        c = 8 * (K - 1 - k) + x;
    }
    const uint8_t *p = buf + (uint64_t)c * kChunk;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = *(const G u32x4 *)(p + (u * 256 + threadIdx.x) * 16);
    if (COPY) {
#pragma unroll
        for (int u = 0; u < 4; u++)
            __builtin_nontemporal_store(v[u], (G u32x4 *)(dst + (uint64_t)c * kChunk + (u * 256 + threadIdx.x) * 16));
    } else {
        u32x4 acc = v[0] + v[1] + v[2] + v[3];
        if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = 1u;
    }
}

int main(int argc, char **argv)
{
    const uint64_t mib = argc > 1 ? atoll(argv[1]) : 16;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    const uint32_t nchunk = (uint32_t)((mib << 20) / kChunk);
    uint8_t *buf;
    uint32_t *owner, *lists, *len, *heads, *sink;
    CHECK(hipMalloc(&buf, (uint64_t)nchunk * kChunk));
    CHECK(hipMalloc(&owner, nchunk * 4));
    CHECK(hipMalloc(&lists, 8 * nchunk * 4));
    CHECK(hipMalloc(&len, 32));
    CHECK(hipMalloc(&heads, 32));
    CHECK(hipMalloc(&sink, 1024));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const uint32_t rgrid = prop.multiProcessorCount * 8;

    // owner map from one W launch (the dispatcher's round-robin is stable launch to launch;
    // checked below)
    wk<0><<<nchunk, 256>>>(buf, owner, 1);
    CHECK(hipDeviceSynchronize());
    std::vector<uint32_t> own(nchunk), own2(nchunk);
    CHECK(hipMemcpy(own.data(), owner, nchunk * 4, hipMemcpyDeviceToHost));
    wk<0><<<nchunk, 256>>>(buf, owner, 2);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(own2.data(), owner, nchunk * 4, hipMemcpyDeviceToHost));
    uint32_t stable = 0;
    for (uint32_t i = 0; i < nchunk; i++) stable += own[i] == own2[i];
    std::vector<uint32_t> L(8 * nchunk), n(8, 0);
    for (uint32_t i = 0; i < nchunk; i++) L[own[i] * nchunk + n[own[i]]++] = i;
    CHECK(hipMemcpy(lists, L.data(), 8 * nchunk * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(len, n.data(), 32, hipMemcpyHostToDevice));

    uint8_t *dst;
    CHECK(hipMalloc(&dst, (uint64_t)nchunk * kChunk));
    uint32_t xmod = 0;
    for (uint32_t i = 0; i < nchunk; i++) xmod += own[i] == i % 8;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    // R variant v: -1 = none (W alone); else shift = v & 0xFF, rev = v & 0x100, copy = v & 0x200
    auto timeit = [&](int v) {
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int i = 0; i < iters; i++) {
            wk<0><<<nchunk, 256>>>(buf, owner, i);
            if (v < 0) continue;
            if (v & 0x200) rs<true><<<nchunk, 256>>>(buf, dst, nchunk, v & 0xFF, (v & 0x100) != 0, sink);
            else rs<false><<<nchunk, 256>>>(buf, dst, nchunk, v & 0xFF, (v & 0x100) != 0, sink);
        }
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        return ms * 1000.0f / iters;
    };
    timeit(0);
    const float w = timeit(-1);
    printf("{\"MiB\": %llu, \"chunks\": %u, \"owner_stable\": %u, \"owner_is_b_mod_8\": %u, \"us_W\": %.2f",
           (unsigned long long)mib, nchunk, stable, xmod, w);
    const int vs[] = {0, 1, 2, 4, 8, 0x100, 0x200, 0x201, 0x204, 0x300};
    const char *nm[] = {"read_s0", "read_s1", "read_s2", "read_s4", "read_s8", "read_rev",
                        "copy_s0", "copy_s1", "copy_s4", "copy_rev"};
    for (int k = 0; k < 10; k++) {
        const float t1 = timeit(vs[k]), t2 = timeit(vs[k]);
        printf(", \"us_R_%s\": [%.2f, %.2f]", nm[k], t1 - w, t2 - w);
    }
    printf("}\n");
    return 0;
}
