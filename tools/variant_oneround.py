#!/usr/bin/env python3
"""A/B source variant (round 5): the fused reas_kernel for small slots (<= 4 KiB, the
768-thread launch) in ONE copy round -- every thread issues all U of its 16-byte loads
before the classification and stores them after it -- instead of U = 4 in 1.8 software-
pipelined rounds.  The group size follows from the one-round budget NT x U chunks.
Jumbo slots keep the product form (U = 4, 512 threads, pipelined rounds).

  tools/variant_oneround.py NAME U [NT_SMALL]  -> build/variants/src_NAME/ (then hipcc)
"""
import os
import shutil
import subprocess
import sys

name, U = sys.argv[1], int(sys.argv[2])
nt = int(sys.argv[3]) if len(sys.argv) > 3 else 768
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


def sub(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new)


sub("constexpr int kReasU = 4;", "constexpr int kReasU = 4;\nconstexpr int kReasUOne = %d;" % U)
# the copy rounds: one-round form when U != 4 (the small-slot launch)
sub("""    constexpr uint32_t RS = (uint32_t)(NT * U);
    if (RS < nch) issue(RS, y);""", """    constexpr uint32_t RS = (uint32_t)(NT * U);
    if constexpr (U != 4) {
        (void)y;
        store(0u, x);
        for (uint32_t r0 = RS; r0 < nch; r0 += RS) {     // only for a fixed group size past NT x U
            issue(r0, x);
            store(r0, x);
        }
    } else {
    if (RS < nch) issue(RS, y);""")
sub("""        store(r0 + RS, x);
    }
""", """        store(r0 + RS, x);
    }
    }
""")
sub("constexpr int kReasNTSmall = 768;", "constexpr int kReasNTSmall = %d;" % nt)
# group size: the small launch's budget is its one round
sub("""    const uint32_t spc = stride >> 4, budget = kReasChunksPerBlock;
    uint32_t G = 64;
    while (G > 1 && G * spc > budget) G >>= 1;""", """    const uint32_t spc = stride >> 4,
                   budget = NT == kReasNTSmall ? (uint32_t)(kReasUOne * kReasNTSmall) : kReasChunksPerBlock;
    uint32_t G = 64;
    while (G > 1 && G * spc > budget) G >>= 1;
    if (NT == kReasNTSmall) G = budget / spc < 64u ? (budget / spc ? budget / spc : 1u) : 64u;""")
sub("if (c > 64 || 4u * c < 3u * G0 || 3u * c > 4u * G0) continue;",
    "if (c > 64 || c * spc > budget || 4u * c < 3u * G0 || 3u * c > 4u * G0) continue;")
sub("""    const uint32_t cap = NT == kReasNTSmall ? reas_resident_groups<U, kReasNTSmall>()""",
    """    const uint32_t cap = NT == kReasNTSmall ? reas_resident_groups<kReasUOne, kReasNTSmall>()""")
sub("""        hipLaunchKernelGGL((reas_kernel<U, kReasNTSmall>), dim3(groups), dim3(kReasNTSmall), 0, stream, R,""",
    """        hipLaunchKernelGGL((reas_kernel<kReasUOne, kReasNTSmall>), dim3(groups), dim3(kReasNTSmall), 0, stream, R,""")
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
    elif cur and "reas_kernel" in cur and any(k in line for k in ("VGPRs:", "Occupancy", "ScratchSize")):
        print(cur[:48], line.split("remark:")[1].split("[-R")[0].strip())
print("built lib_%s.so" % name)
