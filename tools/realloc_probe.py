"""Config 3's two speeds: does the scatter's mode follow the allocations?

One process allocates P datagram buffers and A reassemblers (each with an event arena of its
own, allocated by the library) and times config 3's batch (70 x 8 MiB at MTU 9000, 65,730
datagrams, 590 MB of slots) for every (buffer, arena) pair: segment, then reassemble_batch
(classify + scatter with streaming loads inside), HIP events around each, the arena
recycled between trials.  A mode that belongs to one buffer or one arena shows up as a row
or a column; a mode of the process as every pair alike.  Prints one JSON line per pair, then
a summary line.
Usage: python tools/realloc_probe.py [--buffers 4] [--arenas 4] [--trials 3]
"""
import argparse
import json
import os
import statistics as st
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from e2sar_amd import sar  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buffers", type=int, default=4)
    ap.add_argument("--arenas", type=int, default=4)
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--events", type=int, default=70)
    ap.add_argument("--event-bytes", type=int, default=8 << 20)
    ap.add_argument("--mtu", type=int, default=9000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = sar.Context(0)
    E, B = a.events, a.event_bytes
    src = torch.empty(E * B, dtype=torch.uint8, device=dev)
    src.random_(0, 256)
    seg = sar.DeviceSegmenter(ctx, mtu=a.mtu)
    plan = seg.plan([(src.data_ptr() + k * B, B, k, 4321, 1 + k, (1 << 48) + k) for k in range(E)])
    n, stride = plan.total_packets, seg.stride
    pks = [torch.empty(n * stride, dtype=torch.uint8, device=dev) for _ in range(a.buffers)]
    ln = torch.empty(n, dtype=torch.int32, device=dev)
    Rs = [sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=4096, queue_capacity=4096,
                                arena_bytes=E * (B + 256) + (64 << 20)) for _ in range(a.arenas)]
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    grid = {}
    for i, pk in enumerate(pks):
        for j, R in enumerate(Rs):
            seg_us, reas_us = [], []
            for t in range(a.trials + 1):
                R.recycle(force=True)
                ev[0].record(s)
                seg.segment(plan, pk, ln)
                ev[1].record(s)
                R.reassemble(pk, stride, ln, n)
                ev[2].record(s)
                torch.cuda.synchronize()
                recs = R.poll()
                if t:
                    seg_us.append(round(ev[0].elapsed_time(ev[1]) * 1000, 1))
                    reas_us.append(round(ev[1].elapsed_time(ev[2]) * 1000, 1))
            ok = len(recs) == E and int(R.stats().errorFlags) == 0
            grid[(i, j)] = st.median(reas_us)
            print(json.dumps({"buffer": i, "arena": j, "pk_va_mod_2M": pk.data_ptr() % (2 << 20),
                              "pk_va": hex(pk.data_ptr()), "arena_va": hex(R.arena_ptr),
                              "arena_va_mod_2M": R.arena_ptr % (2 << 20), "seg_us": seg_us,
                              "reas_us": reas_us, "events_ok": ok}), flush=True)
    rows = {i: round(st.median(grid[(i, j)] for j in range(a.arenas)), 1) for i in range(a.buffers)}
    cols = {j: round(st.median(grid[(i, j)] for i in range(a.buffers)), 1) for j in range(a.arenas)}
    print(json.dumps({"summary": "median reassemble_batch us", "by_buffer": rows, "by_arena": cols}), flush=True)


if __name__ == "__main__":
    main()
