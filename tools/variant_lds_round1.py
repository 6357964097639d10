#!/usr/bin/env python3
"""A/B source variant (round 5): the fused reas_kernel's second copy round loaded into LDS by
LDS-DMA (global_load_lds_dwordx4: no VGPRs held) while wave 0 classifies, beside round 0 in
registers.  At 768 threads the kernel is register-bound at two workgroups per CU, so the
round's 48 KiB of LDS per workgroup costs no occupancy (round 4's slab kernel took every
round through LDS at 256 threads and lost to its occupancy).  After the classification:
wait for both rounds, stores of round 0 from registers, round 1 read back from LDS and
stored.  Rounds past the second (groups above 2 x NT x U chunks) keep the register loop.

  tools/variant_lds_round1.py NAME   -> build/variants/lib_NAME.so
"""
import os
import shutil
import subprocess
import sys

name = sys.argv[1]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "e2sar_amd/csrc")
dst = os.path.join(root, "build/variants/src_" + name)
shutil.rmtree(dst, ignore_errors=True)
os.makedirs(dst)
for f in os.listdir(src):
    if f.endswith((".hip", ".hpp", ".cpp")):
        shutil.copy(os.path.join(src, f), dst)
p = os.path.join(dst, "sar_kernels.hip")
s = open(p).read()


def sub(old, new, cnt=1):
    global s
    assert s.count(old) == cnt, (old[:60], s.count(old))
    s = s.replace(old, new)


# reas_range gets the LDS round buffer
sub("""                                           const uint32_t *__restrict__ lens, uint32_t g0, uint32_t gn, uint64_t now,
                                           uint32_t g, ReasGroupLds &L)
{""", """                                           const uint32_t *__restrict__ lens, uint32_t g0, uint32_t gn, uint64_t now,
                                           uint32_t g, ReasGroupLds &L, u32x4 *ldsR1 = nullptr)
{""")
# after issue(0u, x): LDS-DMA of round 1
sub("""    issue(0u, x);

    unsigned long long old = 0;""", """    issue(0u, x);
    constexpr uint32_t RS1 = (uint32_t)(NT * U);
    const bool r1lds = NT == 768 && RS1 < nch;                      // workgroup-uniform
    if constexpr (NT == 768) if (r1lds) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint32_t i = RS1 + (uint32_t)u * NT + tx;
            asm volatile("" : "+v"(i));       // keep the store pass from reusing this split
            uint32_t p, c;
            split_chunk(i, p, c);
            const uint32_t a = __shfl(gPhase, (int)p), plen = __shfl(gPlen, (int)p);
            uint32_t off = 0, sh;
            if (i < nch && 16u * c < a + plen && (a & 3u) == 0u) off = p * stride + da_window(c, a, hl, stride, sh);
            // M0 = this wave's 1 KiB of the round; lane writes 16 B at M0 + lane * 16
            __builtin_amdgcn_global_load_lds((const E2SAR_GLOBAL void *)(bpk + off),
                                             (__attribute__((address_space(3))) void *)(ldsR1 + (uint32_t)u * NT + (tx & ~63u)),
                                             16, 0, 0);
        }
    }

    unsigned long long old = 0;""")
sub("""    constexpr uint32_t RS = (uint32_t)(NT * U);
    if (RS < nch) issue(RS, y);
    store(0u, x);
    for (uint32_t r0 = RS; r0 < nch; r0 += 2 * RS) {""", """    constexpr uint32_t RS = (uint32_t)(NT * U);
    if constexpr (NT == 768) {
        // only loads are outstanding here (round 0 into x, round 1 into LDS): wait for all
        if (r1lds) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        store(0u, x);
        if (r1lds) {
#pragma unroll
            for (int u = 0; u < U; u++) x[u] = ldsR1[(uint32_t)u * NT + tx];
            store(RS, x);
        }
        for (uint32_t r0 = 2 * RS; r0 < nch; r0 += RS) {             // rounds past the second
            issue(r0, x);
            store(r0, x);
        }
    } else {
    if (RS < nch) issue(RS, y);
    store(0u, x);
    for (uint32_t r0 = RS; r0 < nch; r0 += 2 * RS) {""")
sub("""        if (r0 + 2 * RS < nch) issue(r0 + 2 * RS, y);
        store(r0 + RS, x);
    }
""", """        if (r0 + 2 * RS < nch) issue(r0 + 2 * RS, y);
        store(r0 + RS, x);
    }
    }
""")
# reas_group passes it on; reas_kernel allocates it for the small-slot launch
sub("""                                           uint32_t g, ReasGroupLds &L, const uint32_t *__restrict__ starts = nullptr)
{""", """                                           uint32_t g, ReasGroupLds &L, const uint32_t *__restrict__ starts = nullptr,
                                           u32x4 *ldsR1 = nullptr)
{""")
sub("""    reas_range<U, HO, NT>(R, pkts, stride, lens, g0, gn, now, g, L);""",
    """    reas_range<U, HO, NT>(R, pkts, stride, lens, g0, gn, now, g, L, ldsR1);""")
sub("""    __shared__ ReasGroupLds L;
    reas_group<U, false, NT>(R, pkts, stride, lens, n, now, G, blockIdx.x, L, starts);""",
    """    __shared__ ReasGroupLds L;
    __shared__ u32x4 r1[NT == 768 ? NT * U : 1];
    reas_group<U, false, NT>(R, pkts, stride, lens, n, now, G, blockIdx.x, L, starts, NT == 768 ? r1 : nullptr);""")
open(p, "w").write(s)
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Iinclude", "-I" + dst,
       "-shared", "-o", os.path.join(root, "build/variants/lib_%s.so" % name),
       p, os.path.join(dst, "capi.cpp")]
subprocess.run(cmd, check=True, cwd=root)
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only",
                    "-Iinclude", "-I" + dst, "-c", p, "-o", "/tmp/_v.o", "-Rpass-analysis=kernel-resource-usage"],
                   cwd=root, capture_output=True, text=True)
cur = None
for line in r.stderr.splitlines():
    if "Function Name:" in line:
        cur = line.split("Function Name:")[1].strip().split()[0]
    elif cur and "reas_kernel" in cur and any(k in line for k in ("VGPRs:", "Occupancy", "ScratchSize", "LDS Size")):
        print(cur[:48], line.split("remark:")[1].split("[-R")[0].strip())
print("built lib_%s.so" % name)
