#!/usr/bin/env python3
"""A/B source variant (round 5): the order in which reas_scatter_kernel's workgroups visit
the batch.  Product: workgroup b takes group b, so the ~2,000 resident workgroups copy one
contiguous ~18 MB stretch of slots into one or two 8 MiB events at a time (config 3).
Variant: S interleaved streams -- workgroup b takes group (b mod S) * F + b / S (F = nb / S,
the first S * F groups; the rest in order), so the groups in flight at any moment are
spread over S stretches of the whole batch and every event.

  tools/variant_scatter_order.py NAME S   -> build/variants/lib_NAME.so
"""
import os
import shutil
import subprocess
import sys

name, S = sys.argv[1], int(sys.argv[2])
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
old = """    __shared__ PktInfo sinfo[64];
    scatter_group<U, NT, STAGE>(R, pkts, stride, n, G, info, fin, blockIdx.x, sinfo);"""
new = """    __shared__ PktInfo sinfo[64];
    constexpr uint32_t S = %du;
    const uint32_t nb = (n + G - 1u) / G, F = nb / S, b = blockIdx.x;
    const uint32_t blk = (b < S * F) ? (b %% S) * F + b / S : b;
    scatter_group<U, NT, STAGE>(R, pkts, stride, n, G, info, fin, blk, sinfo);""" % S
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Iinclude", "-I" + dst,
       "-shared", "-o", os.path.join(root, "build/variants/lib_%s.so" % name),
       p, os.path.join(dst, "capi.cpp")]
subprocess.run(cmd, check=True, cwd=root)
print("built lib_%s.so" % name)
