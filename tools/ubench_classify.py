#!/usr/bin/env python3
"""Where the classification time goes: one 128 x 1 MiB batch (MTU 1500) classified on a
fresh table (every event created: claim + allocate + publish), then classified again
(every event found: lookup only), then scattered; HIP-event times per launch."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from e2sar_amd import sar
    dev = torch.device("cuda", 0)
    ctx = sar.Context(0)
    B, BE = 1 << 20, int(sys.argv[1]) if len(sys.argv) > 1 else 128
    seg = sar.DeviceSegmenter(ctx, mtu=1500)
    evs = (B + 255) // 256 * 256
    src = torch.randint(0, 256, (BE, evs), dtype=torch.uint8, device=dev)
    plan = seg.plan([(src[i].data_ptr(), B, i, 4321, 1 + i, (1 << 48) + i) for i in range(BE)])
    n = plan.total_packets
    pk, ln = seg.alloc_packets(n)
    seg.segment(plan, pk, ln)
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=4096, queue_capacity=4096,
                              arena_bytes=2 * BE * evs + 4096)
    w = R.alloc_work(n)
    s = torch.cuda.current_stream()
    res = {"create": [], "lookup": [], "scatter": [], "fused_create": [], "fused_lookup": []}
    for it in range(5):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
        R.recycle(force=True)
        e[0].record(s)
        R.classify(pk, seg.stride, ln, n, w)
        e[1].record(s)
        R.classify(pk, seg.stride, ln, n, w)
        e[2].record(s)
        R.scatter(pk, seg.stride, n, w)
        e[3].record(s)
        R.recycle(force=True)
        e[4].record(s)
        R.reassemble(pk, seg.stride, ln, n)
        e[5].record(s)
        R.reassemble(pk, seg.stride, ln, n)
        e[6].record(s)
        torch.cuda.synchronize()
        if it == 0:
            continue
        res["create"].append(e[0].elapsed_time(e[1]) * 1e3)
        res["lookup"].append(e[1].elapsed_time(e[2]) * 1e3)
        res["scatter"].append(e[2].elapsed_time(e[3]) * 1e3)
        res["fused_create"].append(e[4].elapsed_time(e[5]) * 1e3)
        res["fused_lookup"].append(e[5].elapsed_time(e[6]) * 1e3)
    out = {k: round(sum(v) / len(v), 1) for k, v in res.items()}
    out["unit"] = "us per launch"
    out["batch"] = f"{BE} x 1 MiB, MTU 1500, {n} datagrams"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
