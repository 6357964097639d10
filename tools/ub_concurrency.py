#!/usr/bin/env python3
"""Experiment: what running segmentation and reassembly concurrently could buy.

Times one step of the bench workload (E x B events in batches) three ways:
  serial     seg(b) -> reas(b) on one stream (what bench.py does)
  twostream  seg(b) on stream 0 and reas of pre-segmented batch b on stream 1, no
             dependencies between the streams (an upper bound for overlapping the two)
  segonly / reasonly   each chain alone
Usage: python tools/ub_concurrency.py [--events 1024 --batch 128 --mtu 1500]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from e2sar_amd import sar  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mtu", type=int, default=1500)
    ap.add_argument("--event-bytes", type=int, default=1 << 20)
    ap.add_argument("--events", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    ctx = sar.Context(0)
    dev = ctx.torch_device
    B, E = a.event_bytes, a.events
    ev_stride = (B + 255) // 256 * 256
    src = torch.randint(0, 256, (E, ev_stride), dtype=torch.uint8, device=dev)
    seg = sar.DeviceSegmenter(ctx, mtu=a.mtu)
    plans = [seg.plan([(src[i].data_ptr(), B, i, 4321, 1 + i, (1 << 48) + i) for i in range(b0, min(E, b0 + a.batch))])
             for b0 in range(0, E, a.batch)]
    npk = max(p.total_packets for p in plans)
    work = seg.alloc_packets(npk)
    pre = [seg.alloc_packets(npk) for _ in plans]
    for p, (pk, ln) in zip(plans, pre):
        seg.segment(p, pk, ln)
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=4096, queue_capacity=E + 64,
                              lost_capacity=1024, arena_bytes=E * ev_stride + 4096)
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()

    def serial():
        R.recycle(force=True)
        for p in plans:
            seg.segment(p, *work)
            R.reassemble(work[0], seg.stride, work[1], p.total_packets)

    def segonly():
        for p in plans:
            seg.segment(p, *work)

    def reasonly():
        R.recycle(force=True)
        for p, (pk, ln) in zip(plans, pre):
            R.reassemble(pk, seg.stride, ln, p.total_packets)

    def twostream():
        R.recycle(force=True)
        s1.wait_stream(s0)
        for p, (pk, ln) in zip(plans, pre):
            seg.segment(p, *work, stream=s0)
            R.reassemble(pk, seg.stride, ln, p.total_packets, stream=s1)
        s0.wait_stream(s1)

    out = {}
    for name, fn in (("serial", serial), ("segonly", segonly), ("reasonly", reasonly), ("twostream", twostream),
                     ("serial2", serial)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        out[name] = {"ms_per_step": round(ms, 4), "GiB_s": round(E * B / (ms / 1e3) / 2**30, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
