// Which XCD runs workgroup b?  (round 5, config 3's visit order)
// The scatter forms give XCD (b mod 8) runs of consecutive groups, assuming the dispatcher
// deals workgroups round-robin over the 8 XCDs.  This probe records HW_REG_XCC_ID per
// workgroup for grids shaped like the scatter's (256 threads, config 3: 65,730 workgroups;
// headline split: 18,271), with uneven per-workgroup work so dispatch happens under load,
// and reports how many workgroups sit on XCD (b + c) mod 8 for the best c, per launch.
// Run it in several processes: a process-dependent dispatch would show here.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_xcc.hip -o build/ubench_xcc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(256) void xcc_kernel(uint32_t *xcc, uint32_t spin)
{
    __shared__ uint32_t pad[4096];                       // 16 KiB of LDS: occupancy like the staged scatter
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    pad[threadIdx.x] = x;
    // uneven work: blocks whose index hashes low spin longer
    const uint32_t h = (blockIdx.x * 2654435761u) >> 28;
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)spin * (1u + h % 4u)) __builtin_amdgcn_s_sleep(1);
    __syncthreads();
    if (threadIdx.x == 0) xcc[blockIdx.x] = pad[(threadIdx.x + 1) & 255] & 0xF;
}

int main()
{
    const uint32_t grids[] = {65730, 18271, 4096, 1000};
    uint32_t *d = nullptr;
    hipMalloc(&d, 65730 * sizeof(uint32_t));
    std::vector<uint32_t> h(65730);
    printf("{\"launches\": [");
    bool first = true;
    for (uint32_t spin : {0u, 20u}) {
        for (uint32_t n : grids) {
            hipMemset(d, 0xFF, n * sizeof(uint32_t));
            hipLaunchKernelGGL(xcc_kernel, dim3(n), dim3(256), 0, 0, d, spin);
            hipDeviceSynchronize();
            hipMemcpy(h.data(), d, n * sizeof(uint32_t), hipMemcpyDeviceToHost);
            uint32_t best = 0, bestc = 0, per[8] = {0};
            for (uint32_t c = 0; c < 8; c++) {
                uint32_t m = 0;
                for (uint32_t b = 0; b < n; b++) m += (h[b] == ((b + c) & 7u));
                if (m > best) best = m, bestc = c;
            }
            for (uint32_t b = 0; b < n; b++) if (h[b] < 8) per[h[b]]++;
            printf("%s{\"grid\": %u, \"spin_ticks\": %u, \"round_robin_matches\": %u, \"offset\": %u, \"first16\": [",
                   first ? "" : ", ", n, spin, best, bestc);
            for (int i = 0; i < 16; i++) printf("%s%u", i ? "," : "", h[i]);
            printf("], \"per_xcc\": [");
            for (int i = 0; i < 8; i++) printf("%s%u", i ? "," : "", per[i]);
            printf("]}");
            first = false;
        }
    }
    printf("]}\n");
    hipFree(d);
    return 0;
}
