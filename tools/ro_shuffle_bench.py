#!/usr/bin/env python3
"""Reference-order reassembly under reordered arrival (round 5).

One batch of E events of B bytes is segmented on the device; then every event's datagrams
after its first (offset 0 stays first, so every event still completes under the
reference's rules) are shuffled within windows of W datagrams, W = 1 being arrival in
order and W = 0 a full shuffle of the event; and groups of K events are interleaved
datagram by datagram (round robin, each event's own order kept), K = 1 being one event
after another -- K concurrent senders.  The mode's cost follows the runs of one event in
arrival order (K = 205 makes every run one datagram long).  The batch is reassembled with
E2SAR_HIP_REAS_REFERENCE_ORDER and timed with HIP events; every event is checked complete
and byte-exact against its source.

  python tools/ro_shuffle_bench.py [--events 205] [--event-bytes 1048576] [--mtu 1500]
                                   [--windows 1,8,64,0] [--interleave 1] [--reps 5]
Prints one JSON line per (window, interleave).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=205)
    ap.add_argument("--event-bytes", type=int, default=1 << 20)
    ap.add_argument("--mtu", type=int, default=1500)
    ap.add_argument("--windows", default="1,8,64,0")
    ap.add_argument("--interleave", default="1")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--extra-flags", type=lambda v: int(v, 0), default=0,
                    help="e2sar_hip_reas_config.flags bits OR'd in (e.g. 4: E2SAR_HIP_REAS_COLD_DATAGRAMS)")
    args = ap.parse_args()

    import torch
    from e2sar_amd import sar, _capi

    dev = torch.device("cuda:0")
    ctx = sar.Context(0)
    E, B = args.events, args.event_bytes
    seg = sar.DeviceSegmenter(ctx, mtu=args.mtu, lb_hdr_version=2)
    stride = seg.stride
    npk = sar.num_packets(B, seg.max_pld)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    ev_stride = (B + 255) // 256 * 256
    src = torch.randint(0, 256, (E, ev_stride), dtype=torch.uint8, device=dev, generator=g)
    plan = seg.plan([(src[i].data_ptr(), B, i, 4321, 1 + i, (1 << 48) + i) for i in range(E)])
    n = plan.total_packets
    assert n == E * npk
    pk, ln = seg.alloc_packets(n)
    seg.segment(plan, pk, ln)
    torch.cuda.synchronize()
    table = 1
    while table < 8 * E:
        table <<= 1
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=table, queue_capacity=E + 64,
                              lost_capacity=1024, arena_bytes=E * ev_stride + 4096,
                              flags=_capi.REAS_REFERENCE_ORDER | args.extra_flags)
    pk2, ln2 = seg.alloc_packets(n)
    algo = E * (2 * B + 36 * npk)
    cases = [(int(w), int(k)) for w in args.windows.split(",") for k in args.interleave.split(",")]
    for w, K in cases:
        # per event: datagram 0 first, the rest permuted within windows of w (0: all of them)
        body = torch.arange(1, npk, device=dev)
        keys = torch.rand((E, npk - 1), device=dev, generator=g)
        if w == 1:
            perm = body.expand(E, -1)
        else:
            blk = (body - 1) // (w if w > 0 else npk)
            perm = torch.argsort(blk.expand(E, -1).to(torch.float64) * 4 + keys.to(torch.float64), dim=1) + 1
        order = torch.cat([torch.zeros((E, 1), dtype=torch.int64, device=dev), perm], dim=1)
        order = order + torch.arange(E, device=dev).unsqueeze(1) * npk          # [E, npk] positions
        # groups of K events, round robin datagram by datagram
        parts = []
        for e0 in range(0, E, K):
            parts.append(order[e0:e0 + K].t().reshape(-1))
        order = torch.cat(parts)
        pk2.view(-1, stride)[:n] = pk.view(-1, stride)[order]
        ln2[:n] = ln[order]
        evo = order // npk                                    # event of each arrival position
        runs = int((evo[1:] != evo[:-1]).sum().item()) + 1    # runs of one event in arrival order
        times = []
        for rep in range(args.reps + 1):
            R.recycle(force=True)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(int(2e6))
            e0.record()
            R.reassemble(pk2, stride, ln2, n, now_ms=100)
            e1.record()
            torch.cuda.synchronize()
            if rep:
                times.append(e0.elapsed_time(e1) * 1e3)
            recs = R.poll()
            ok = len(recs) == E and all(r.numFragments == npk and r.bytes == B for r in recs)
            if ok and rep == args.reps:
                arena = R.arena_tensor()
                for r in recs:
                    if not torch.equal(arena[r.arenaOffset:r.arenaOffset + B], src[r.eventNum, :B]):
                        ok = False
                        break
            if not ok:
                break
        st = R.stats()
        us = sorted(times)[len(times) // 2] if times else None
        print(json.dumps({"window": w, "interleave": K, "events": E, "event_bytes": B, "mtu": args.mtu, "datagrams": n,
                          "event_runs_in_arrival_order": runs, "us_per_batch_median": round(us, 1) if us else None,
                          "us_all": [round(t, 1) for t in times],
                          "GiB_per_s": round(E * B / (us * 1e-6) / 2**30, 1) if us else None,
                          "achieved_GBps": round(algo / (us * 1e-6) / 1e9, 1) if us else None,
                          "verified": ok, "dataErrCnt": int(st.dataErrCnt), "errorFlags": int(st.errorFlags)}),
              flush=True)
        if not ok:
            sys.exit(1)


if __name__ == "__main__":
    main()
