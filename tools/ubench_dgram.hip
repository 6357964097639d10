// ubench_dgram.hip -- the copy half of config 3's reassembly, isolated: a seg-like kernel W
// writes a buffer of datagram slots (16 KiB per workgroup, streaming source loads, plain
// stores), then a copy kernel R moves it to a destination with non-temporal loads and
// stores.  R variants:
//   lin16 / lin8      : plain copy, 16-KiB / 8-KiB pieces (U = 4 / 2 chunks per thread)
//   dg<G>             : the scatter's pattern -- G slots of `stride` bytes per workgroup,
//                       slot p's payload [36, 36 + pld) to dst + p * pld (misaligned 16-B
//                       stores when pld is not a multiple of 16), chunks spread over the
//                       256 threads in rounds of 256 x U
//   dga<G>            : the same with destination-aligned stores (each lane loads the two
//                       source chunks its aligned destination chunk needs)
// Usage: ubench_dgram [MiB] [stride] [pld] [iters]   -> one JSON line (µs of R)
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

__global__ __launch_bounds__(256) void wk(const uint8_t *src, uint8_t *mid, uint64_t bytes)
{
    const uint64_t base = (uint64_t)blockIdx.x * 16384;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint64_t i = base + (u * 256 + threadIdx.x) * 16;
        v[u] = i + 16 <= bytes ? ldnt(src + i) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint64_t i = base + (u * 256 + threadIdx.x) * 16;
        if (i + 16 <= bytes) *(G u32x4 *)(mid + i) = v[u] + 1u;
    }
}

template <int U>
__global__ __launch_bounds__(256) void lin(const uint8_t *mid, uint8_t *dst, uint64_t bytes)
{
    const uint64_t base = (uint64_t)blockIdx.x * (256 * 16 * U);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t i = base + (u * 256 + threadIdx.x) * 16;
        v[u] = i + 16 <= bytes ? ldnt(mid + i) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t i = base + (u * 256 + threadIdx.x) * 16;
        if (i + 16 <= bytes) stnt(dst + i, v[u]);
    }
}

__device__ __forceinline__ u32x4 funnel(u32x4 a, u32x4 b, uint32_t s)   // bytes [s, s+16) of a:b
{
    uint32_t c0, c1, c2, c3, c4;
    switch (s >> 2) {
    case 0: c0 = a.x; c1 = a.y; c2 = a.z; c3 = a.w; c4 = b.x; break;
    case 1: c0 = a.y; c1 = a.z; c2 = a.w; c3 = b.x; c4 = b.y; break;
    case 2: c0 = a.z; c1 = a.w; c2 = b.x; c3 = b.y; c4 = b.z; break;
    default: c0 = a.w; c1 = b.x; c2 = b.y; c3 = b.z; c4 = b.w; break;
    }
    const uint32_t r = s & 3u;
    return u32x4{__builtin_amdgcn_alignbyte(c1, c0, r), __builtin_amdgcn_alignbyte(c2, c1, r),
                 __builtin_amdgcn_alignbyte(c3, c2, r), __builtin_amdgcn_alignbyte(c4, c3, r)};
}

__device__ __forceinline__ uint8_t byte_of(u32x4 v, int k)     // k a constant after unrolling
{
    return (uint8_t)(v[k >> 2] >> (8 * (k & 3)));
}

// source-aligned: chunk c of slot p (c >= 2 covers payload bytes); store its payload bytes at
// their destination, 16-B store when all 16 are payload (misaligned), dword / byte stores at the edges
template <int U, bool ALIGNED>
__global__ __launch_bounds__(256) void dg(const uint8_t *mid, uint8_t *dst, uint32_t nslots, uint32_t stride,
                                          uint32_t pld, uint32_t Gs, uint32_t H, uint32_t force)
{
    const uint32_t p0 = blockIdx.x * Gs;
    const uint32_t gn = nslots - p0 < Gs ? nslots - p0 : Gs;
    const uint32_t spc = stride / 16;
    if (!ALIGNED) {
        const uint32_t nch = gn * spc;
        for (uint32_t r0 = 0; r0 < nch; r0 += 256 * U) {
            u32x4 x[U];
            uint32_t pp[U], cc[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t i = r0 + u * 256 + threadIdx.x, ic = i < nch ? i : 0;
                pp[u] = ic / spc;
                cc[u] = ic - pp[u] * spc;
                x[u] = ldnt(mid + (uint64_t)(p0 + pp[u]) * stride + 16 * cc[u]);
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t i = r0 + u * 256 + threadIdx.x;
                if (i >= nch) continue;
                const int64_t s0 = (int64_t)16 * cc[u] - H;            // payload byte of the chunk's first byte
                if (s0 >= (int64_t)pld || s0 + 16 <= 0) continue;
                uint8_t *D = dst + (uint64_t)(p0 + pp[u]) * pld;
                if (s0 >= 0 && s0 + 16 <= (int64_t)pld) {
                    // misaligned 16-B store (4-B aligned when pld % 4 == 0)
                    uint32_t *d4 = (uint32_t *)(D + s0);
                    if (force) d4 = (uint32_t *)((uintptr_t)d4 & ~(uintptr_t)15);   // perf probe: wrong bytes
                    if ((((uintptr_t)d4) & 15u) == 0) stnt((uint8_t *)d4, x[u]);
                    else {
                        typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(4)));
                        __builtin_nontemporal_store(*(u32x4u *)&x[u], (G u32x4u *)d4);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 16; k++) {
                        const int64_t t = s0 + k;
                        if (t >= 0 && t < (int64_t)pld) D[t] = byte_of(x[u], k);
                    }
                }
            }
        }
    } else {
        // destination chunks: slot p's payload occupies dst bytes [p*pld, p*pld+pld); work in
        // aligned 16-B destination blocks, each lane loading the source bytes it needs
        const uint64_t d0 = (uint64_t)p0 * pld, d1 = (uint64_t)(p0 + gn) * pld;
        const uint64_t a0 = d0 & ~15ull;
        const uint32_t nblk = (uint32_t)((d1 - a0 + 15) / 16);
        for (uint32_t r0 = 0; r0 < nblk; r0 += 256 * U) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t k = r0 + u * 256 + threadIdx.x;
                if (k >= nblk) continue;
                const uint64_t db = a0 + 16ull * k;                        // dst byte of the block
                const uint64_t lo = db < d0 ? d0 : db, hi = db + 16 > d1 ? d1 : db + 16;
                // slot of the block's first payload byte; a block may straddle two slots
                const uint32_t p = (uint32_t)(lo / pld);
                const uint64_t off = lo - (uint64_t)p * pld;               // payload byte in slot p
                const uint64_t sb = (uint64_t)p * stride + 36 + off - (lo - db);   // src byte for dst byte db
                const uint64_t sa = sb & ~15ull;
                const u32x4 A = ldnt(mid + sa), B = ldnt(mid + sa + 16);
                u32x4 o = funnel(A, B, (uint32_t)(sb - sa));
                const bool whole = lo == db && hi == db + 16 && (uint64_t)(p + 1) * pld >= db + 16;
                if (whole) stnt(dst + db, o);
                else {
#pragma unroll
                    for (int k = 0; k < 16; k++) {
                        const uint64_t t = db + k;
                        if (t < lo || t >= hi) continue;
                        const uint32_t q = (uint32_t)(t / pld);
                        dst[t] = q == p ? byte_of(o, k) : mid[(uint64_t)q * stride + 36 + (t - (uint64_t)q * pld)];
                    }
                }
            }
        }
    }
}

int main(int argc, char **argv)
{
    const uint64_t mib = argc > 1 ? atoll(argv[1]) : 560;
    const uint32_t stride = argc > 2 ? atoi(argv[2]) : 8976;
    uint32_t pld = argc > 3 ? atoi(argv[3]) : 8936;
    const int iters = argc > 4 ? atoi(argv[4]) : 10;
    const uint32_t nslots = (uint32_t)((mib << 20) / stride);
    const uint64_t bytes = (uint64_t)nslots * stride;
    uint8_t *src, *mid, *dst;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&mid, bytes));
    CHECK(hipMalloc(&dst, bytes));
    CHECK(hipMemset(src, 0x5a, bytes));
    const uint32_t wgrid = (uint32_t)((bytes + 16383) / 16384);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    uint32_t H = 36, force = 0;
    auto timeit = [&](int v, uint32_t Gs) {
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int i = 0; i < iters; i++) {
            wk<<<wgrid, 256>>>(src, mid, bytes);
            switch (v) {
            case 0: break;
            case 1: lin<4><<<(uint32_t)((bytes + 16383) / 16384), 256>>>(mid, dst, bytes); break;
            case 2: lin<2><<<(uint32_t)((bytes + 8191) / 8192), 256>>>(mid, dst, bytes); break;
            case 3: dg<4, false><<<(nslots + Gs - 1) / Gs, 256>>>(mid, dst, nslots, stride, pld, Gs, H, force); break;
            case 4: dg<8, false><<<(nslots + Gs - 1) / Gs, 256>>>(mid, dst, nslots, stride, pld, Gs, H, force); break;
            case 5: dg<4, true><<<(nslots + Gs - 1) / Gs, 256>>>(mid, dst, nslots, stride, pld, Gs, H, force); break;
            case 6: dg<8, true><<<(nslots + Gs - 1) / Gs, 256>>>(mid, dst, nslots, stride, pld, Gs, H, force); break;
            }
        }
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        CHECK(hipGetLastError());
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        return ms * 1000.0f / iters;
    };
    timeit(1, 1);
    const float w = timeit(0, 1);
    printf("{\"MiB\": %llu, \"stride\": %u, \"pld\": %u, \"us_W\": %.2f", (unsigned long long)(bytes >> 20), stride, pld, w);
    struct V { const char *nm; int v; uint32_t g; };
    const V vs[] = {{"lin16", 1, 1}, {"lin8", 2, 1}, {"dg1_u4", 3, 1}, {"dg2_u4", 3, 2}, {"dg2_u8", 4, 2},
                    {"dg3_u8", 4, 3}, {"dga1_u4", 5, 1}, {"dga2_u8", 6, 2}, {"dg8_u4", 3, 8}, {"dg11_u4", 3, 11}};
    for (const V &x : vs) {
        if (x.g * (stride / 16) > 8192) continue;
        const float t1 = timeit(x.v, x.g), t2 = timeit(x.v, x.g);
        printf(", \"us_R_%s\": [%.2f, %.2f]", x.nm, t1 - w, t2 - w);
    }
    // the same one-slot pattern with the payload 16-B aligned in the slot (H = 48), and with
    // every 16-B store forced to an aligned address (perf probe only: wrong bytes)
    const uint32_t Gbest = stride >= 4096 ? 1 : 8;
    H = 48;
    printf(", \"us_R_dg_H48\": %.2f", timeit(3, Gbest) - w);
    force = 1;
    printf(", \"us_R_dg_H48_forcealign\": %.2f", timeit(3, Gbest) - w);
    H = 36;
    printf(", \"us_R_dg_H36_forcealign\": %.2f", timeit(3, Gbest) - w);
    force = 0;
    // the one-slot geometry with nothing skipped or shifted (whole slots to dst + p * stride):
    // what the workgroup shape alone costs against lin8 / lin16
    H = 0;
    const uint32_t pld0 = pld;
    pld = stride;
    printf(", \"us_R_slotcopy_g1_u4\": %.2f", timeit(3, 1) - w);
    printf(", \"us_R_slotcopy_g%u_u4\": %.2f", Gbest == 1 ? 2 : Gbest, timeit(3, Gbest == 1 ? 2 : Gbest) - w);
    pld = pld0;
    H = 36;
    printf("}\n");
    return 0;
}
