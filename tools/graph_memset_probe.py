#!/usr/bin/env python3
"""Probe: hipMemsetAsync nodes of several sizes captured into a HIP graph, each followed by
kernels that read the zeroed range, replayed three times.  Prints one line
per size as it goes, so a fault names the size it happened at."""
import ctypes as C
import sys

import torch

hiprt = C.CDLL("libamdhip64.so")
hiprt.hipMemsetAsync.restype = C.c_int
hiprt.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]

for size in [int(x) for x in sys.argv[1:]] or [4, 8, 4096, 1 << 20, 1228800, 16 << 20]:
    n = size // 4
    buf = torch.ones(n + 64, dtype=torch.int32, device="cuda")
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())

    def body(stream):
        assert hiprt.hipMemsetAsync(C.c_void_p(buf.data_ptr()), 0, size, C.c_void_p(int(stream.cuda_stream))) == 0
        return buf[:n].sum(), buf[n:].sum()

    with torch.cuda.stream(cap):
        body(cap)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        zs, gs = body(cap)
    ok = True
    seen = []
    for r in range(3):
        buf.fill_(1)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        seen.append((int(zs), int(gs), int((buf[:n] != 0).sum())))
        ok &= int(zs) == 0 and int(gs) == 64
    print(f"memset {size} B captured, 3 replays: {'ok' if ok else 'WRONG'} "
          f"(sum of zeroed range, guard sum, nonzero words per replay: {seen})", flush=True)
    del g
    torch.cuda.synchronize()
sys.exit(0)
