#!/usr/bin/env python3
"""Timeline of one seg_kernel + reas_kernel launch pair (experiment build with -DE2SAR_TRACE=1).

Runs the bench's default batch (205 x 1 MiB events, MTU 1500) a few times, then records
per-workgroup s_memrealtime stamps of one more pair and prints where the time goes:
launch span, dispatch ramp, classification latency, store phase and the tail.
Usage: E2SAR_HIP_LIB=build/variants/lib_trace.so python tools/trace_reas.py [--mtu M --event-bytes B --batch N]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from e2sar_amd import sar  # noqa: E402
from e2sar_amd._capi import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mtu", type=int, default=1500)
    ap.add_argument("--event-bytes", type=int, default=1 << 20)
    ap.add_argument("--batch", type=int, default=205)
    ap.add_argument("--out", default="")
    ap.add_argument("--standalone", action="store_true",
                    help="reassemble a batch segmented earlier, after 1.5 GB of other traffic (cold datagrams)")
    a = ap.parse_args()
    L = lib()
    L.e2sar_hip_debug_trace.argtypes = [C.c_int, C.c_void_p, C.c_size_t]
    ctx = sar.Context(0)
    dev = ctx.torch_device
    B, E = a.event_bytes, a.batch
    ev_stride = (B + 255) // 256 * 256
    src = torch.randint(0, 256, (E, ev_stride), dtype=torch.uint8, device=dev)
    seg = sar.DeviceSegmenter(ctx, mtu=a.mtu)
    plan = seg.plan([(src[i].data_ptr(), B, i, 4321, 1 + i, (1 << 48) + i) for i in range(E)])
    pk, ln = seg.alloc_packets(plan.total_packets)
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=4096, queue_capacity=E + 64,
                              lost_capacity=1024, arena_bytes=E * ev_stride + 4096)
    for _ in range(4):
        R.recycle(force=True)
        seg.segment(plan, pk, ln)
        R.reassemble(pk, seg.stride, ln, plan.total_packets)
    torch.cuda.synchronize()
    L.e2sar_hip_debug_trace_clear()
    R.recycle(force=True)
    torch.cuda.synchronize()
    seg.segment(plan, pk, ln)
    if a.standalone:
        junk = torch.empty(3 << 29, dtype=torch.uint8, device=dev)
        junk.fill_(1)
        del junk
    R.reassemble(pk, seg.stride, ln, plan.total_packets)
    torch.cuda.synchronize()
    out = {}
    for k, name in ((1, "seg"), (0, "reas")):
        buf = np.zeros(16384 * 4, np.uint64)
        assert L.e2sar_hip_debug_trace(k, buf.ctypes.data, buf.size) == 0
        t = buf.reshape(-1, 4)
        t = t[t[:, 0] != 0]
        out[name] = t
    t0 = min(int(out["seg"][:, 0].min()), int(out["reas"][:, 0].min()))
    res = {}
    for name, t in out.items():
        st = (t[:, 0].astype(np.int64) - t0) * 10 / 1000.0        # 100 MHz ticks -> us
        en = t[:, 3].astype(np.int64)
        ok = en != 0
        en = (en - t0) * 10 / 1000.0
        hw = t[:, 2]
        xcc = (hw >> np.uint64(32)) & np.uint64(0xF)
        r = {
            "blocks": int(len(t)),
            "first_start_us": float(st.min()), "last_start_us": float(st.max()),
            "start_q": [float(x) for x in np.quantile(st, [0.1, 0.5, 0.9])],
            "end_q": [float(x) for x in np.quantile(en[ok], [0.1, 0.5, 0.9, 1.0])],
            "dur_q": [float(x) for x in np.quantile((en - st)[ok], [0.1, 0.5, 0.9])],
            "blocks_per_xcc": np.bincount(xcc.astype(np.int64), minlength=8).tolist(),
        }
        if name == "reas":
            cl = (t[:, 1].astype(np.int64) - t[:, 0].astype(np.int64)) * 10 / 1000.0
            r["classify_q"] = [float(x) for x in np.quantile(cl, [0.1, 0.5, 0.9, 1.0])]
            # classification detail (k = 2): header loads back, first CAS back, lookup done, passes
            d = np.zeros(16384 * 4, np.uint64)
            assert L.e2sar_hip_debug_trace(2, d.ctypes.data, d.size) == 0
            d = d.reshape(-1, 4)[: len(t)].astype(np.int64)
            s0 = t[:, 0].astype(np.int64)
            okd = (d[:, 0] != 0) & (d[:, 1] != 0) & (d[:, 2] != 0)
            q = lambda v: [round(float(x), 2) for x in np.quantile(v[okd], [0.1, 0.5, 0.9])]
            r["detail_us_q10_50_90"] = {
                "headers": q((d[:, 0] - s0) * 0.01),
                "first_cas": q((d[:, 1] - d[:, 0]) * 0.01),
                "rest_of_lookup": q((d[:, 2] - d[:, 1]) * 0.01),
                "after_lookup": q((t[:, 1].astype(np.int64) - d[:, 2]) * 0.01),
                "passes": q(d[:, 3].astype(np.float64) * 100.0),
            }
            # first-wave blocks only (started within 2 us of the first)
            fw = okd & (st < st.min() + 2.0)
            r["first_wave_blocks"] = int(fw.sum())
            qf = lambda v: [round(float(x), 2) for x in np.quantile(v[fw], [0.1, 0.5, 0.9])]
            r["first_wave_detail"] = {"headers": qf((d[:, 0] - s0) * 0.01), "first_cas": qf((d[:, 1] - d[:, 0]) * 0.01),
                                      "rest_of_lookup": qf((d[:, 2] - d[:, 1]) * 0.01),
                                      "after_lookup": qf((t[:, 1].astype(np.int64) - d[:, 2]) * 0.01)}
            # the groups dispatched later (started 10 us or more after the first)
            lw = okd & (st >= st.min() + 10.0)
            r["later_blocks"] = int(lw.sum())
            if lw.any():
                ql = lambda v: [round(float(x), 2) for x in np.quantile(v[lw], [0.1, 0.5, 0.9])]
                r["later_detail"] = {"headers": ql((d[:, 0] - s0) * 0.01), "first_cas": ql((d[:, 1] - d[:, 0]) * 0.01),
                                     "rest_of_lookup": ql((d[:, 2] - d[:, 1]) * 0.01),
                                     "after_lookup": ql((t[:, 1].astype(np.int64) - d[:, 2]) * 0.01),
                                     "classify": ql(cl)}
        # concurrency profile: running blocks per 2 us bin
        lo, hi = float(st.min()), float(en[ok].max())
        bins = np.arange(lo, hi + 2, 2.0)
        run = [int(((st <= b) & (en > b)).sum()) for b in bins]
        r["running_per_2us"] = run
        res[name] = r
    print(json.dumps(res, indent=1))
    if a.out:
        np.savez(a.out, seg=out["seg"], reas=out["reas"])


if __name__ == "__main__":
    main()
