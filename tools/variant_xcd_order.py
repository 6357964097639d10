#!/usr/bin/env python3
"""A/B source variant (round 5): XCD-aware visit order for the scatter forms.

Workgroup b of a launch runs on XCD b mod 8.  Product: scatter workgroup b takes group b,
so consecutive groups (8 datagrams at MTU 1500, one at 9000) sit on different XCDs and
every group boundary -- a 128-byte line shared by two datagrams' slots and, at the
destination, by two payloads -- is touched by two XCDs' L2s.  Variants remap the logical
group of workgroup b so each XCD walks its own groups:
  S<n>: n regions, workgroup b takes region b mod n at step b / n (n = 8: XCD x streams the
        x-th eighth of the batch);
  K<k>: runs of k consecutive groups per XCD, the eight XCDs' runs side by side, moving
        through the batch together.
Applied to reas_scatter_kernel and to the scatter half of reas_scatter_classify_kernel
(whose classify workgroup count is rounded up to a multiple of 8 so the scatter
workgroups keep their XCD parity).

  tools/variant_xcd_order.py NAME S8|K16|... [fused]   -> build/variants/lib_NAME.so
  (fused: the fused reas_kernel's groups are remapped too)
"""
import os
import shutil
import subprocess
import sys

name, kind = sys.argv[1], sys.argv[2]
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


v = int(kind[1:])
if kind[0] == "S":
    fn = """__device__ __forceinline__ uint32_t xcd_order(uint32_t b, uint32_t nb)
{
    constexpr uint32_t S = %du;
    const uint32_t F = nb / S;
    return (b < S * F) ? (b %% S) * F + b / S : b;
}
""" % v
else:
    fn = """__device__ __forceinline__ uint32_t xcd_order(uint32_t b, uint32_t nb)
{
    constexpr uint32_t K = %du, W = 8u * K;
    if (b >= (nb / W) * W) return b;
    const uint32_t w = b %% W;
    return (b - w) + (w %% 8u) * K + w / 8u;
}
""" % v
sub("__global__ __launch_bounds__(kBlock) void reas_classify_kernel(", fn + "\n__global__ __launch_bounds__(kBlock) void reas_classify_kernel(")
sub("""    __shared__ PktInfo sinfo[64];
    scatter_group<U, NT, STAGE>(R, pkts, stride, n, G, info, fin, blockIdx.x, sinfo);""",
    """    __shared__ PktInfo sinfo[64];
    scatter_group<U, NT, STAGE>(R, pkts, stride, n, G, info, fin, xcd_order(blockIdx.x, (n + G - 1u) / G), sinfo);""")
sub("""    const uint32_t sb = (b < clsStart) ? b : b - nClsBlocks;
    scatter_group<U, NT, STAGE>(R, spk, stride, sn, G, sinfoG, sfin, sb, sinfo);""",
    """    const uint32_t sb = (b < clsStart) ? b : b - nClsBlocks;
    scatter_group<U, NT, STAGE>(R, spk, stride, sn, G, sinfoG, sfin, xcd_order(sb, (sn + G - 1u) / G), sinfo);""")
sub("""    const uint32_t nCls = cdiv(cn, kScatBlock);""", """    const uint32_t nCls = (cdiv(cn, kScatBlock) + 7u) & ~7u;     // keeps the scatter blocks' XCD parity""")
sub("""    const uint32_t clsStart = (uint32_t)((uint64_t)sblocks * kPipeClsAtPercent / 100u);""",
    """    const uint32_t clsStart = (uint32_t)((uint64_t)sblocks * kPipeClsAtPercent / 100u) & ~7u;""")
if len(sys.argv) > 3 and sys.argv[3] == "fused":
    # the fused reas_kernel's groups too
    sub("""    __shared__ ReasGroupLds L;
    reas_group<U, false, NT>(R, pkts, stride, lens, n, now, G, blockIdx.x, L, starts);""",
        """    __shared__ ReasGroupLds L;
    reas_group<U, false, NT>(R, pkts, stride, lens, n, now, G, starts ? blockIdx.x : xcd_order(blockIdx.x, (n + G - 1u) / G), L, starts);""")
    # xcd_order must be declared before reas_kernel
    s = s.replace(fn + "\n__global__ __launch_bounds__(kBlock) void reas_classify_kernel(",
                  "__global__ __launch_bounds__(kBlock) void reas_classify_kernel(")
    sub("// reas_kernel: workgroup b reassembles datagrams", fn + "\n// reas_kernel: workgroup b reassembles datagrams")
open(p, "w").write(s)
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Iinclude", "-I" + dst,
       "-shared", "-o", os.path.join(root, "build/variants/lib_%s.so" % name),
       p, os.path.join(dst, "capi.cpp")]
subprocess.run(cmd, check=True, cwd=root)
print("built lib_%s.so" % name)
