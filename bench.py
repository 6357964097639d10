#!/usr/bin/env python3
"""Benchmark: GiB/s of event payload segmented + reassembled, device-resident, on MI355X.

One step = every event of this rank's working set (default 1024 x 1 MiB) is segmented
into LB+RE datagrams (MTU 1500 -> 731 per event) and the datagrams are reassembled
into a fresh event arena, batch by batch (default 205 events = 149,855 datagrams =
221 MB of datagram slots per batch, so a batch's datagrams can stay in the 256 MiB
Infinity Cache between the two kernels; A/B: 128 -> 1295 GiB/s, 192 -> 1331,
205 -> 1351, 228 -> 1314, 256 -> 1187).  Inputs (event bytes + the 40-byte-per-event descriptor tables) are resident
in HBM before timing starts.  N>1: one process per GPU (torch.distributed.run), events
sharded by eventNum % world (weak scaling, no data-path collective).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mtu", type=int, default=1500)
    ap.add_argument("--event-bytes", type=int, default=1 << 20)
    ap.add_argument("--events", type=int, default=1024, help="events per rank per step")
    ap.add_argument("--batch-events", type=int, default=205,
                    help="events per segment/reassemble launch (205 x 1 MiB: 150K datagrams, 221 MB: five "
                         "launches per 1024-event step whose datagram batch still fits the 256 MiB Infinity Cache)")
    ap.add_argument("--lb-version", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--payload", choices=["random", "perf"], default="random",
                    help="random: seeded uniform bytes; perf: e2sar_perf's event (head 'This is a start of "
                         "event payload', tail '...the end', bin/e2sar_perf.cpp:27-28,153-154; zeros between)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--eager", action="store_true", help="launch from Python each step instead of a HIP graph")
    ap.add_argument("--overlap", action="store_true", help="reassemble batch b while segmenting b+1 (2 streams)")
    ap.add_argument("--reas", choices=["fused", "split", "pipelined"], default="fused",
                    help="fused: one reassemble_batch launch per batch; split: classify + scatter launches "
                         "in line; pipelined: one launch scatters batch b while other workgroups classify "
                         "batch b+1 (two datagram buffers, one stream)")
    ap.add_argument("--roofline-steps", type=int, default=2)
    ap.add_argument("--landing", choices=["own", "spread"], default="own",
                    help="own: datagrams land on their owner; spread: owners spread, RCCL exchange (config 4)")
    ap.add_argument("--table-factor", type=int, default=8,
                    help="event-table slots = next power of two >= factor x events per step")
    ap.add_argument("--quiet", action="store_true")
    return ap.parse_args()


def log(args, *a):
    if not args.quiet:
        print(*a, file=sys.stderr, flush=True)


def cpu_baseline(args, budget_s: float):
    """The oracle (plain-C restatement of _send + recv body) on the host cores, on a bounded
    sample of the same workload: each thread segments + reassembles its own 16 events of
    event-bytes repeatedly.  Timed on 1 thread and on T threads (the box's CPU share,
    OMP_NUM_THREADS, at most 16; ctypes releases the GIL around every C call), budget_s
    each; the T-thread rate is the reported baseline."""
    import threading

    import numpy as np

    import oracle_ffi as O
    import sar_inputs as S

    B = args.event_bytes
    n_ev = max(1, min(16, (256 << 20) // B))
    mp = O.max_pld_len(args.mtu)
    stride = (36 + mp + 15) // 16 * 16
    npk = O.num_packets(B, mp)
    events = [S.event_bytes(i, B) for i in range(n_ev)]

    import ctypes as C

    def worker(deadline, out, idx):
        L = O.lib()
        pk = np.zeros((npk, stride), np.uint8)
        ln = np.zeros(npk, np.uint32)
        evp = C.POINTER(C.c_uint8)()
        nb, en, di = C.c_size_t(), C.c_uint64(), C.c_uint16()
        done = 0
        while True:
            r = O.Reassembler(True, 1 << 20)
            for i, ev in enumerate(events):
                L.e2o_segment_event(ev.ctypes.data, B, i, S.DATA_ID, S.entropy(i), S.lb_tick(i),
                                    args.lb_version, mp, pk.ctypes.data, stride, ln.ctypes.data)
                r.push_batch(pk, ln)
                # getEvent hands the event buffer over and the caller frees it
                # (e2sarDPReassembler.cpp:626-641; delete[] in bin/e2sar_perf.cpp:299)
                assert L.e2o_reas_pop(r.h, C.byref(evp), C.byref(nb), C.byref(en), C.byref(di)) == 0
                assert nb.value == B
                L.e2o_free(evp)
            done += n_ev * B
            del r
            if time.perf_counter() >= deadline:
                break
        out[idx] = done

    def run(threads):
        out = [0] * threads
        t0 = time.perf_counter()
        ts = [threading.Thread(target=worker, args=(t0 + budget_s, out, k)) for k in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        dt = time.perf_counter() - t0
        return sum(out) / dt / 2**30, sum(out) // (n_ev * B), dt

    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    T = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", share)), share))
    v1, p1, d1 = run(1)
    vT, pT, dT = run(T) if T > 1 else (v1, p1, d1)
    what = (f"MTU {args.mtu}: oracle segment_event (header + payload memcpy per datagram) then recv "
            f"body (parse, map lookup, memcpy) into a fresh event handed out like getEvent and freed, "
            f"each thread {n_ev} x {B} B events per pass")
    return {"value": round(vT, 4), "unit": "GiB/s", "cores": T, "kind": "port",
            "sample": f"{pT} passes on {T} threads in {dT:.1f} s; {what}",
            "single_core": {"value": round(v1, 4), "cores": 1, "sample": f"{p1} passes in {d1:.1f} s"}}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from e2sar_amd import sar

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # E2SAR_BENCH_BACKEND=gloo + E2SAR_BENCH_SHARE_GPU=1 rehearse the N>1 flow with every
    # rank on GPU 0 (a one-GPU box); the driver's multi-GPU runs use RCCL ("nccl").
    backend = os.environ.get("E2SAR_BENCH_BACKEND", "nccl")
    if os.environ.get("E2SAR_BENCH_SHARE_GPU") == "1":
        local = 0
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ctx = sar.Context(local)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")

    B = args.event_bytes
    E = args.events
    seg = sar.DeviceSegmenter(ctx, mtu=args.mtu, lb_hdr_version=args.lb_version)
    mp, stride = seg.max_pld, seg.stride
    npk = sar.num_packets(B, mp)

    # ---- inputs resident in HBM: event bytes + per-batch descriptor tables ----
    g = torch.Generator(device=dev)
    g.manual_seed(0xE25A2 + rank)
    ev_stride = (B + 255) // 256 * 256
    src = torch.randint(0, 256, (E, ev_stride), dtype=torch.uint8, device=dev, generator=g)
    if args.payload == "perf":
        head, tail = b"This is a start of event payload", b"...the end"
        assert B >= len(head) + len(tail)
        src.zero_()
        src[:, :len(head)] = torch.tensor(list(head), dtype=torch.uint8, device=dev)
        src[:, B - len(tail):B] = torch.tensor(list(tail), dtype=torch.uint8, device=dev)
    if args.landing == "own":
        evnum = lambda i: i * world + rank      # every local event is owned here: eventNum % world == rank
    else:
        evnum = lambda i: rank * E + i          # owners spread over all ranks: datagrams must be exchanged
    plans = []
    for b0 in range(0, E, args.batch_events):
        idx = range(b0, min(E, b0 + args.batch_events))
        plans.append(seg.plan([(src[i].data_ptr(), B, evnum(i), 4321, 1 + (evnum(i) * 0x9E37) % 65535,
                                (1 << 48) + evnum(i)) for i in idx]))
    max_batch_pk = max(p.total_packets for p in plans)
    if args.reas == "pipelined" and args.overlap:
        args.overlap = False                    # the pipeline is its own overlap
    nbuf = 2 if (args.overlap or args.reas == "pipelined") else 1
    bufs = [seg.alloc_packets(max_batch_pk) for _ in range(nbuf)]
    table = 1
    while table < args.table_factor * E:
        table <<= 1
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=max(table, 64), queue_capacity=E + 64,
                              lost_capacity=1024, arena_bytes=E * ev_stride + 4096)
    works = [R.alloc_work(max_batch_pk) for _ in range(nbuf)] if args.reas != "fused" else None
    torch.cuda.synchronize()

    timing = []          # (kernel, start event, end event) while the roofline pass runs
    timing_on = [False]

    def timed(name, fn, *a, **kw):
        """Launch fn; in the roofline pass bracket it with HIP events on the current stream."""
        if not timing_on[0]:
            return fn(*a, **kw)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fn(*a, **kw)
        e1.record()
        timing.append((name, e0, e1))
        return r

    def reassemble(pk, ln, n, k, stream=None):
        """The receive side of one batch: one fused launch, or classify + scatter."""
        if args.reas == "fused":
            timed("reas_kernel", R.reassemble, pk, stride, ln, n, stream=stream)
        else:
            w = works[k % nbuf]
            timed("reas_classify_kernel", R.classify, pk, stride, ln, n, w, stream=stream)
            timed("reas_scatter_kernel", R.scatter, pk, stride, n, w, stream=stream)

    def step():
        """One step: recycle the event table/arena, then segment -> reassemble every batch.
        With --overlap, reassembly of batch b runs on a second stream concurrently with
        segmentation of batch b+1 (double-buffered datagram slots)."""
        s0 = torch.cuda.current_stream()
        R.recycle(force=True)
        if args.landing == "spread":
            # datagrams land on this rank whatever their owner: route by owner on the GPU,
            # one all-to-all-v over RCCL, reassemble what this rank owns
            pk, ln = bufs[0]
            for p in plans:
                timed("seg_kernel", seg.segment, p, pk, ln)
                spk, sln, cnt = timed("route_kernels", router.route, pk, ln, p.total_packets)
                if world > 1:
                    rpk, rln, n = timed("exchange", dexchange, spk, sln, [int(c) for c in cnt.tolist()], stride)
                else:
                    rpk, rln, n = spk, sln, p.total_packets
                timed("reas_kernel", R.reassemble, rpk, stride, rln, n)
            return
        if args.reas == "pipelined":
            # seg(0), classify(0); then per batch: seg(b+1), [scatter(b) | classify(b+1)]
            # in one launch; buffers b%2 are rewritten by seg(b+2) after that launch.
            n0 = plans[0].total_packets
            timed("seg_kernel", seg.segment, plans[0], *bufs[0])
            timed("reas_classify_kernel", R.classify, bufs[0][0], stride, bufs[0][1], n0, works[0])
            for k, p in enumerate(plans):
                pk, ln = bufs[k % 2]
                if k + 1 < len(plans):
                    q = plans[k + 1]
                    npk_, nln_ = bufs[(k + 1) % 2]
                    timed("seg_kernel", seg.segment, q, npk_, nln_)
                    timed("reas_scatter_classify_kernel", R.scatter_classify, stride, pk, p.total_packets,
                          works[k % 2], npk_, nln_, q.total_packets, works[(k + 1) % 2])
                else:
                    timed("reas_scatter_kernel", R.scatter, pk, stride, p.total_packets, works[k % 2])
            return
        if not args.overlap:
            pk, ln = bufs[0]
            for k, p in enumerate(plans):
                timed("seg_kernel", seg.segment, p, pk, ln)
                reassemble(pk, ln, p.total_packets, k)
            return
        s1 = side
        s1.wait_stream(s0)
        done = [None] * nbuf
        for k, p in enumerate(plans):
            pk, ln = bufs[k % nbuf]
            if done[k % nbuf] is not None:
                s0.wait_event(done[k % nbuf])
            seg.segment(p, pk, ln, stream=s0)
            ev = torch.cuda.Event()
            ev.record(s0)
            s1.wait_event(ev)
            reassemble(pk, ln, p.total_packets, k, stream=s1)
            d = torch.cuda.Event()
            d.record(s1)
            done[k % nbuf] = d
        s0.wait_stream(s1)

    side = torch.cuda.Stream() if args.overlap else None

    router = None
    if args.landing == "spread":
        from e2sar_amd.dist import PacketRouter, exchange as dexchange
        router = PacketRouter(ctx, stride, max_batch_pk, world, rank)
        if args.overlap or not args.eager or args.reas != "fused":
            log(args, "landing=spread: counts are read back per batch -> eager, fused, no overlap")
        args.overlap = False
        args.reas = "fused"
        args.eager = True

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # ---- correctness gate (outside the timed region) ----
    def verify_spread():
        recs = R.poll()
        st = R.stats()
        arena = R.arena_tensor()
        # per-event byte sums of every rank's source events, all-gathered
        sums = src[:, :B].to(torch.int64).sum(dim=1)
        ids = torch.tensor([evnum(i) for i in range(E)], dtype=torch.int64, device=dev)
        table = torch.stack([ids, sums], dim=1)
        if world > 1:
            table = table.to(coll_dev)
            allt = [torch.empty_like(table) for _ in range(world)]
            dist.all_gather(allt, table)
            table = torch.cat(allt).to(dev)
        ref = {int(a): int(b) for a, b in table.tolist()}
        owned = [e for e in ref if e % world == rank]
        ok = (len(recs) == len(owned) and st.inProgress == 0 and st.badHeaderDiscards == 0)
        for r in recs:
            if not ok:
                break
            ok = int(arena[r.arenaOffset: r.arenaOffset + B].to(torch.int64).sum()) == ref.get(r.eventNum, -1)
        if not ok:
            raise SystemExit(f"rank {rank}: spread-landing verification FAILED ({len(recs)} records)")
        return True

    def verify():
        if args.landing == "spread":
            return verify_spread()
        recs = R.poll()
        st = R.stats()
        arena = R.arena_tensor()
        ok = (len(recs) == E and st.inProgress == 0 and st.badHeaderDiscards == 0
              and all(r.numFragments == npk for r in recs))
        if ok:
            for r in recs:
                i = (r.eventNum - rank) // world
                if not torch.equal(arena[r.arenaOffset: r.arenaOffset + B], src[i, :B]):
                    ok = False
                    break
        if not ok:
            raise SystemExit(f"rank {rank}: round-trip verification FAILED ({len(recs)} records, stats "
                             f"eventSuccess={st.eventSuccess} inProgress={st.inProgress})")
        return True

    verified = None
    if not args.no_verify:
        step()
        torch.cuda.synchronize()
        verified = verify()

    # ---- the step as one HIP graph (kills per-launch host overhead) ----
    graph = None
    if not args.eager:
        graph = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream()
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            step()                          # warm the capture stream once
        torch.cuda.synchronize()
        with torch.cuda.graph(graph, stream=cap):
            step()
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        if not args.no_verify:
            verified = verify() and verified is not False

    # ---- timed region ----
    K = args.steps
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        if graph is not None:
            graph.replay()
        else:
            step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- per-kernel durations: HIP events around each launch of the step, eager, on the
    # stream the kernels run on (the step is single-stream unless --overlap) ----
    was_overlap = args.overlap
    args.overlap = False
    timing_on[0] = True
    for _ in range(max(1, args.roofline_steps)):
        step()
    torch.cuda.synchronize()
    timing_on[0] = False
    args.overlap = was_overlap
    per = {}
    for name, e0, e1 in timing:
        per.setdefault(name, []).append(e0.elapsed_time(e1))
    avg = {k: sum(v) / len(v) for k, v in per.items()}
    per_launch_events = sum(p.n_events for p in plans) / len(plans)
    # algorithmic bytes of one launch of each bandwidth kernel:
    #   seg: B + (B + 36N) per event; reassembly (fused, scatter, scatter+classify): (B + 36N) + B
    #   (the classify share of scatter+classify -- 24 B of header/length read and 16 B of
    #   record written per datagram -- is left out, so its rate is understated by ~1 %)
    launch_bytes = per_launch_events * (2 * B + 36 * npk)
    bw_kernels = [k for k in avg if k in ("seg_kernel", "reas_kernel", "reas_scatter_kernel",
                                          "reas_scatter_classify_kernel")]
    dom = max(bw_kernels, key=lambda k: sum(per[k]))      # most time in the step
    dom_ms = avg[dom]
    achieved = launch_bytes / (dom_ms * 1e-3) / 1e9

    # HBM traffic per launch of the dominant kernel, from the committed rocprofv3 PMC passes
    # of this same workload (tools/pmc_summary.py; FETCH_SIZE x2 + WRITE_SIZE, gfx950 rules)
    traffic = None
    traffic_src = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            w = pmc.get("workload") or {}
            if (w.get("mtu") == args.mtu and w.get("event_bytes") == B and w.get("batch_events") == args.batch_events
                    and w.get("lb_version", 2) == args.lb_version):
                for k, v in pmc["kernels"].items():
                    if k.startswith(dom):
                        traffic = int(v["hbm_bytes_per_launch"])
                        traffic_src = pmc.get("file", "profiles/round1/final/pmc_summary.json")
        except (OSError, ValueError, KeyError):
            traffic = None

    total_payload = E * B * world * K
    value = total_payload / elapsed / 2**30
    step_bytes = E * (4 * B + 72 * npk)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(args, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "GiB/s event payload segmented+reassembled, device-resident, 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": ("synthetic (torch Philox uniform bytes, seeded per rank)" if args.payload == "random" else
                     "synthetic (e2sar_perf event pattern: head + tail strings, zeros between)"),
            "config": {
                "workload": (f"{E} x {B} B events/rank/step, MTU {args.mtu} (maxPld {mp}, {npk} datagrams/event), "
                             f"LB v{args.lb_version} + RE headers, withLBHeader, {args.batch_events} events per "
                             f"launch, segment -> reassemble in HBM"),
                "events_per_rank": E, "event_bytes": B, "mtu": args.mtu, "batch_events": args.batch_events,
                "table_slots": max(table, 64),
                "parallelism": (f"eventNum % {world} sharding (no collective)" if args.landing == "own" else
                                f"eventNum % {world} owners, datagrams land spread: route + all-to-all-v "
                                f"({backend}) + reassemble"),
                "launch": "eager" if args.eager else "hipGraph per step",
                "overlap": bool(args.overlap),
                "reassembly": {"fused": "reas_kernel per batch",
                               "split": "reas_classify_kernel + reas_scatter_kernel per batch",
                               "pipelined": "reas_scatter_classify_kernel: scatter(b) beside classify(b+1), "
                                            "2 datagram buffers"}[args.reas],
                "landing": args.landing,
                "payload": args.payload,
                "verified_roundtrip": verified,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_unit": "bytes per launch (rocprofv3 PMC, committed)" if traffic else None,
                "traffic_source": traffic_src,
                "avg_launch_ms": {k: round(v, 5) for k, v in avg.items()},
                "launches_per_step": {k: len(v) // max(1, args.roofline_steps) for k, v in per.items()},
                "algorithmic_bytes_per_launch": int(launch_bytes),
                "step_achieved_GBps": round(step_bytes * K / elapsed / 1e9, 1),
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
