#!/usr/bin/env python3
"""Benchmark: GiB/s of event payload segmented + reassembled, device-resident, on MI355X.

One step = every event of this rank's working set (default 1024 x 1 MiB) is segmented
into LB+RE datagrams (MTU 1500 -> 731 per event) and the datagrams are reassembled
into a fresh event arena, batch by batch (default 205 events = 149,855 datagrams =
221 MB of datagram slots per batch, so a batch's datagrams can stay in the 256 MiB
Infinity Cache between the two kernels; A/B: 128 -> 1295 GiB/s, 192 -> 1331,
205 -> 1351, 228 -> 1314, 256 -> 1187).  Inputs (event bytes + the 40-byte-per-event
descriptor tables) are resident in HBM before timing starts.

N>1: one process per GPU.  `python bench.py --gpus N` started without WORLD_SIZE starts
`torch.distributed.run --nproc-per-node N` itself (a child process, before any GPU call)
and exits with its status; every rank checks WORLD_SIZE == --gpus.  Events are sharded
by eventNum % world (weak scaling, no data-path collective); `--landing spread` adds the
route + all-to-all-v exchange of config 4.

A second, separately reported leg (`reas_cold`) times the receive side alone on
datagrams written long before (every batch in its own buffer, 1.1 GB in all, so each
launch reads them back from HBM, not from the Infinity Cache): the real receive path.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

BEST_COPY_GBS = 6240.0
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec
XGMI_PEAK_GBS = 7 * 153.0  # per GPU, 7 xGMI links x ~153 GB/s (point to point)
METRIC = "GiB/s event payload segmented+reassembled, device-resident, 1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--warm-timed", type=int, default=1,
                    help="1: repeat the warmup steps (as the timed steps run: graph replays) right before "
                         "the timed region's barrier; 0: only before verification and capture")
    ap.add_argument("--mtu", type=int, default=1500)
    ap.add_argument("--event-bytes", type=int, default=1 << 20)
    ap.add_argument("--events", type=int, default=1024, help="events per rank per step")
    ap.add_argument("--batch-events", type=int, default=205,
                    help="events per segment/reassemble launch (205 x 1 MiB: 150K datagrams, 221 MB: five "
                         "launches per 1024-event step whose datagram batch still fits the 256 MiB Infinity Cache)")
    ap.add_argument("--lb-version", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget per thread count (0 = skip)")
    ap.add_argument("--payload", choices=["random", "perf"], default="random",
                    help="random: seeded uniform bytes; perf: e2sar_perf's event (head 'This is a start of "
                         "event payload', tail '...the end', bin/e2sar_perf.cpp:27-28,153-154; zeros between)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--eager", action="store_true", help="launch from Python each step instead of a HIP graph")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="steps captured in one HIP graph (0: all --steps in one graph, up to 64; above that "
                         "the largest divisor of --steps up to 64); "
                         "the timed region still runs exactly --steps steps")
    ap.add_argument("--overlap", action="store_true", help="reassemble batch b while segmenting b+1 (2 streams)")
    ap.add_argument("--xcd-groups", type=int, default=0,
                    help="1: reassemble each batch over the group table that matches seg_kernel's XCD stripes "
                         "(e2sar_hip_seg_groups / e2sar_hip_reassemble_groups: every datagram read on the XCD "
                         "that wrote it)")
    ap.add_argument("--guided", default="",
                    help="A/B: 'F,SMIN,RESIDENT' guided group sizes for the fused reassembly (see run_workload)")
    ap.add_argument("--lanes", type=int, default=1,
                    help="independent segment -> reassemble pipelines on this many streams, batches dealt out "
                         "round-robin, each lane with its own datagram buffer (so the datagrams resident at "
                         "once stay lanes x batch): one lane's launch head and tail overlap another's body")
    ap.add_argument("--reas", choices=["fused", "split", "pipelined", "chained"], default="fused",
                    help="fused: one reassemble_batch launch per batch; split: classify + scatter launches "
                         "in line; pipelined: one launch scatters batch b while other workgroups classify "
                         "batch b+1 (two datagram buffers, one stream); chained: segmentation and "
                         "reassembly of a batch in one launch (segment_reassemble_batch)")
    ap.add_argument("--reference-order", action="store_true",
                    help="reassemble with E2SAR_HIP_REAS_REFERENCE_ORDER (the reference's arrival-order rules: "
                         "key pass, radix sort, per-key walk, scatter)")
    ap.add_argument("--chain-batches", type=int, default=1,
                    help="chained form: batches per launch (1-8; each batch its own datagram buffer)")
    ap.add_argument("--roofline-steps", type=int, default=2)
    ap.add_argument("--landing", choices=["own", "spread"], default="own",
                    help="own: datagrams land on their owner; spread: owners spread, RCCL exchange (config 4)")
    ap.add_argument("--fold-recycle", type=int, default=1,
                    help="1: the step's table/arena recycle runs inside its first seg_kernel launch "
                         "(e2sar_hip_segment_batch_recycle); 0: a reas_recycle_kernel launch of its own")
    ap.add_argument("--reas-group", type=int, default=0,
                    help="A/B: datagrams per fused-reassembly workgroup (1..64; 0 = the library's balanced choice)")
    ap.add_argument("--table-factor", type=int, default=8,
                    help="event-table slots = next power of two >= factor x events per step")
    ap.add_argument("--cold-steps", type=int, default=10,
                    help="steps of the cold receive-only leg (0 = skip): reassembly of datagrams that were "
                         "written long before and are read back from HBM")
    ap.add_argument("--cold-batch-events", type=int, default=0,
                    help="events per reassembly launch in the cold leg (0 = every event of the step in one "
                         "classify and one scatter launch); the cold leg does not depend on the Infinity "
                         "Cache holding a batch, so larger launches only amortise a launch's head and tail "
                         "(round 5: split form, 1024 / 512 / 205 events: 2552-2564 / 2471 / 2278-2293 GiB/s; "
                         "pipelined 205 / 512: 2418-2444 / 2522-2527)")
    ap.add_argument("--cold-reas", choices=["fused", "split", "pipelined"], default="split",
                    help="launch form of the cold leg (split: classify + scatter launches, timed apart; "
                         "pipelined: classify(0), then scatter(b) beside classify(b+1) in one launch)")
    ap.add_argument("--subs", default="auto",
                    help="sub-legs reported beside the headline (comma list of mtu9000, config3, spread; "
                         "'none' to skip; 'auto' = mtu9000,config3 at N=1 and spread at N>1): north_star's "
                         "MTU 9000 half (1 MiB events), BASELINE config 3 (8 MiB events at MTU 9000, 70 "
                         "events = 65,730 datagrams per launch) and BASELINE config 4 (datagrams landing "
                         "spread over the ranks, exchanged over RCCL)")
    ap.add_argument("--quiet", action="store_true")
    return ap.parse_args(argv)


def log(args, *a):
    if not args.quiet:
        print(*a, file=sys.stderr, flush=True)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args) -> int:
    """`--gpus N` without a launcher: run this script under torch.distributed.run as a child
    process (nothing here has touched the GPU) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def host_cpu_info() -> dict:
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = os.cpu_count() or 1
    return {"nproc": os.cpu_count(), "allowed": allowed, "model": model}


# per-thread datagram ring and live-event window of the CPU baseline's DRAM-streaming form
CPU_RING_BYTES = 64 << 20


def cpu_baseline(args, budget_s: float):
    """The oracle (plain-C restatement of _send + recv body) on the host cores, on a bounded
    sample of the same workload: each thread segments + reassembles the sample's events
    (64 x 1 MiB by default) repeatedly, budget_s per thread count.  Three thread counts:
    1; T = the GPU's share of the host (the CPUs this process may use, capped at 16: the
    GPU box allots 16 host CPUs per GPU, OMP_NUM_THREADS=16 there) -- the reported `value`;
    and every CPU this process may use (`all_cores`, sched_getaffinity = nproc on the box),
    SURVEY 8(d)'s nproc figure.  The threads are POSIX threads inside the oracle library
    (oracle/cpu_bench.c), so no interpreter lock sits between them.

    Working set: every figure but `cache_resident` streams from DRAM -- each thread
    segments into a ring of 64 MiB of datagram buffers and keeps its last 64 MiB of
    reassembled events alive (CPU_RING_BYTES), as the GPU's 1 GiB step streams from HBM.
    `cache_resident` is the earlier form (one datagram buffer and one reused event block
    per thread, L2/L3-resident: superlinear in threads), at 1 and T threads, half the
    budget each, for comparison."""
    import ctypes as C

    import numpy as np

    import oracle_ffi as O
    import sar_inputs as S

    B = args.event_bytes
    # events in the sample (E2SAR_CPU_EVENTS overrides): 64 MiB of events, more than a
    # CCD's 32 MB L3, so one thread streams them from DRAM as 16 threads do (and as the GPU
    # workload's 1 GiB does).  A 4-16 MiB sample runs one thread from its L3 at ~1.7x the
    # DRAM rate, which is why an earlier 16-event sample showed 16 threads at only 1.3-2.6x
    # one (tools/cpu_baseline_sweep.sh)
    n_ev = int(os.environ.get("E2SAR_CPU_EVENTS", 0)) or max(1, min(64, (64 << 20) // B))
    mp = O.max_pld_len(args.mtu)
    sample = np.concatenate([S.event_bytes(i, B) for i in range(n_ev)])
    L = O.lib()

    def run(threads, ring=CPU_RING_BYTES, seconds=budget_s):
        done, dt = C.c_uint64(), C.c_double()
        rc = L.e2o_cpu_bench(sample.ctypes.data, n_ev, B, args.lb_version, mp, S.DATA_ID, threads,
                             seconds, ring, C.byref(done), C.byref(dt))
        if rc != 0:
            raise RuntimeError(f"oracle CPU baseline failed on {threads} threads")
        return done.value / dt.value / 2**30, done.value // (n_ev * B), dt.value

    info = host_cpu_info()
    omp = int(os.environ.get("OMP_NUM_THREADS", info["allowed"]))
    T = max(1, min(16, omp, info["allowed"]))
    v1, p1, d1 = run(1)
    vT, pT, dT = run(T) if T > 1 else (v1, p1, d1)
    A = info["allowed"]
    vA, pA, dA = run(A) if A > T else (vT, pT, dT)
    c1, q1, e1 = run(1, 0, budget_s / 2)
    cT, qT, eT = run(T, 0, budget_s / 2) if T > 1 else (c1, q1, e1)
    what = (f"MTU {args.mtu}: oracle segment_event (header + payload memcpy per datagram) then recv "
            f"body (parse, map lookup, memcpy) into a fresh event handed out like getEvent, "
            f"each thread {n_ev} x {B} B events per pass")
    ring_mib = CPU_RING_BYTES >> 20
    ws = (f"streams from DRAM: the shared {n_ev * B >> 20} MiB event sample, plus per thread a {ring_mib} MiB ring "
          f"of datagram buffers and its last {ring_mib} MiB of reassembled events kept alive (freed oldest first)")
    return {"value": round(vT, 4), "unit": "GiB/s", "cores": T, "kind": "port",
            "sample": f"{pT} passes on {T} threads in {dT:.1f} s; {what}",
            "working_set": ws,
            "host": {**info, "threads_used": T,
                     "cap": "min(16, OMP_NUM_THREADS, sched_getaffinity): the GPU box's CPU share per GPU"},
            "single_core": {"value": round(v1, 4), "cores": 1, "sample": f"{p1} passes in {d1:.1f} s"},
            "all_cores": {"value": round(vA, 4), "cores": A, "sample": f"{pA} passes on {A} threads in {dA:.1f} s",
                          "note": "every CPU sched_getaffinity allows this process (the whole host on the GPU box, "
                                  "shared with the other GPUs' jobs)"},
            "cache_resident": {"value": round(cT, 4), "cores": T, "single_core": round(c1, 4),
                               "sample": f"{qT} passes on {T} threads in {eT:.1f} s, {q1} on 1 in {e1:.1f} s",
                               "working_set": "each thread reuses one datagram buffer and one event block (freed "
                                              "before the next is allocated, so malloc returns the same block): "
                                              "only the shared event sample streams from DRAM; L2/L3-resident "
                                              "otherwise, hence superlinear in threads"},
            "config1_loopback": cpu_loopback(args, min(5.0, budget_s))}


def cpu_loopback(args, seconds: float):
    """BASELINE config 1 (bin/e2sar_perf loopback on the host CPU, one Segmenter and one
    Reassembler thread): oracle/build/e2o_loopback -- the oracle's SAR path with one sendto
    per datagram and one recvfrom per datagram over UDP 127.0.0.1, the sender keeping at most
    half a receive buffer of datagrams in flight (the fastest lossless rate)."""
    exe = os.path.join(ROOT, "oracle", "build", "e2o_loopback")
    if not os.path.exists(exe):
        return None
    try:
        out = subprocess.run([exe, str(args.event_bytes), str(args.mtu), str(seconds)], capture_output=True,
                             text=True, timeout=seconds + 30)
        res = json.loads(out.stdout.strip().splitlines()[-1])
    except (OSError, ValueError, IndexError, subprocess.TimeoutExpired):
        return None
    res["what"] = ("1 segmenter thread + 1 reassembler thread, UDP loopback, sendto/recvfrom per datagram, "
                   "oracle segment/receive body; threads 2 (kind port)")
    return res


def graph_steps(args) -> int:
    """Steps captured in one HIP graph.  Default: the whole timed region in one graph (up to 64
    steps; above that the largest divisor of --steps up to 64).  Every graph launch costs the
    GPU idle time at its start (the host submits its nodes), so fewer, longer graphs measure
    the kernels rather than the launches: K = 20 with warm-timed replays, 20-step graph
    1491-1495 GiB/s, 10-step 1450-1464, 4-step 1431-1443, 1-step 1397-1416; K = 200 in
    4-step graphs 1496 (profiles/round6/timed_start/)."""
    if args.graph_steps > 0:
        if args.steps % args.graph_steps:
            raise SystemExit("--steps must be a multiple of --graph-steps")
        return args.graph_steps
    return next(d for d in range(min(args.steps, 64), 0, -1) if args.steps % d == 0)

def _pmc_traffic(args, dom, batch_events=None):
    """HBM traffic per launch of kernel `dom` from the committed rocprofv3 PMC summaries
    (tools/pmc_summary.py; FETCH_SIZE x2 + WRITE_SIZE, gfx950 rules) whose workload is this
    one: profiles/pmc_latest.json and profiles/pmc_*.json.  batch_events: the events per
    launch of the leg asking (the cold leg launches its own batch, not --batch-events)."""
    be = args.batch_events if batch_events is None else batch_events
    import glob
    for path in [os.path.join(ROOT, "profiles", "pmc_latest.json")] + sorted(
            glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))):
        try:
            with open(path) as f:
                pmc = json.load(f)
        except (OSError, ValueError):
            continue
        w = pmc.get("workload") or {}
        if (w.get("mtu") == args.mtu and w.get("event_bytes") == args.event_bytes
                and w.get("batch_events") == be and w.get("lb_version", 2) == args.lb_version):
            ks = pmc.get("kernels") or {}
            # reassemble_batch's split form (batches above 320 MiB of slots) is two launches
            parts = ("reas_classify_kernel", "reas_scatter_kernel") if dom == "reassemble_batch_split" else (dom,)
            got = [v for p in parts for k, v in ks.items() if k.split("<")[0] == p]
            if len(got) == len(parts):
                return int(sum(v["hbm_bytes_per_launch"] for v in got)), pmc.get("file", os.path.relpath(path, ROOT))
    return None, None


def copy_calibration(ctx, torch, dev):
    """Achievable HBM on this device beside the 8 TB/s peak: the best of
    device copies with e2sar_hip_copy_spans (16-byte non-temporal loads and stores, one
    8-KiB piece per workgroup) of uniform random bytes (the headline's payload; constant
    bytes copy faster) at 1 GiB and 4 GiB, read + write bytes per second, HIP events
    around 5 copies each.  The larger copy amortises the launch's head and tail, so the
    fraction of copy the bench reports is taken against the best copy it measured, not a
    flattering one (tools/ubench_store.hip: the best plain copy form measured, 8-KiB
    pieces with nt loads and stores, 6.06 / 6.21 TB/s at 1 / 4 GiB)."""
    best, per = 0.0, {}
    for nb in (1 << 30, 4 << 30):
        a = torch.empty(nb, dtype=torch.uint8, device=dev)
        b = torch.empty(nb, dtype=torch.uint8, device=dev)
        a.random_(0, 256)
        span = [(a.data_ptr(), b.data_ptr(), nb)]
        for _ in range(2):
            ctx.copy_spans(span)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record()
        for _ in range(5):
            ctx.copy_spans(span)
        c1.record()
        torch.cuda.synchronize()
        g = 2 * nb * 5 / (c0.elapsed_time(c1) * 1e-3) / 1e9
        per[f"{nb >> 30}GiB"] = round(g, 1)
        best = max(best, g)
        del a, b
    torch.cuda.empty_cache()
    return best, per


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))

    import torch
    import torch.distributed as dist

    from e2sar_amd import sar

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE {world}: launch one rank per GPU")
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
    env = Env(torch=torch, dist=dist, sar=sar, ctx=ctx, dev=dev, world=world, rank=rank, backend=backend,
              coll_dev=dev if backend == "nccl" else torch.device("cpu"))

    line = run_workload(args, env, headline=True)

    # the other half of north_star's target and BASELINE config 3, in the same run: each a
    # workload of its own (fresh buffers), its own roofline; `value` above stays config 2's
    subs = sub_legs(args, world)
    for name in subs:
        over = SUB_LEGS[name]
        a = argparse.Namespace(**{**vars(args), **over, "cold_steps": 0, "cpu_seconds": 0.0})
        t0 = time.perf_counter()
        # At N > 1 a sub-leg runs collectives (the spread leg's RCCL all-to-alls): should one
        # fail or stall, the headline measured above is still reported -- rank 0 prints its
        # line with the sub-leg's error and every rank exits (os._exit: a rank stuck in a
        # collective cannot return) once the deadline passes
        guard = None
        if world > 1:
            deadline = float(os.environ.get("E2SAR_SUBLEG_DEADLINE_S", "420"))
            guard = threading.Timer(deadline, _abandon_sub_leg, args=(line, name, rank, f"no result in {deadline:.0f} s"))
            guard.daemon = True
            guard.start()
        try:
            sl = run_workload(a, env, headline=False)
        except Exception as e:                  # noqa: BLE001 -- reported, not swallowed
            if world == 1:
                raise
            _abandon_sub_leg(line, name, rank, f"{type(e).__name__}: {e}"[:400])
        if guard is not None:
            guard.cancel()
        torch.cuda.empty_cache()
        if rank == 0:
            line[name] = {
                "workload": sl["config"]["workload"], "value": sl["value"], "unit": sl["unit"],
                "ms_per_step": sl["ms_per_step"], "steps": sl["steps"], "verified": sl["config"]["verified_roundtrip"],
                "reassembly": sl["config"]["reassembly"], "launch": sl["config"]["launch"],
                "roofline": sl["roofline"], "leg_seconds": round(time.perf_counter() - t0, 1)}
            if name == "spread":
                line[name].update({"parallelism": sl["config"]["parallelism"], "xgmi": sl["xgmi"],
                                   "exchange": sl["spread"]})

    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        line["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    if rank == 0:
        _print_line(line)
    if world > 1:
        dist.destroy_process_group()


_LINE_LOCK = threading.Lock()
_LINE_PRINTED = [False]


def _print_line(line):
    """Rank 0's one JSON line, printed once: the deadline timer's thread and the main
    thread may both reach here."""
    with _LINE_LOCK:
        if _LINE_PRINTED[0]:
            return
        _LINE_PRINTED[0] = True
        print(json.dumps(line), flush=True)


def _abandon_sub_leg(line, name: str, rank: int, why: str):
    """A sub-leg at N > 1 failed or stalled: rank 0 prints the run's line (the headline and
    the sub-legs done so far) with this one's error; every rank ends here with status 3, so
    torchrun and CI see the failure (the headline in the line stays readable)."""
    if rank == 0:
        with _LINE_LOCK:
            if not _LINE_PRINTED[0]:
                line[name] = {"error": why}
        _print_line(line)
    sys.stderr.write(f"bench: rank {rank}: sub-leg {name} abandoned ({why})\n")
    sys.stderr.flush()
    os._exit(3)


def sub_legs(args, world: int):
    """The sub-legs of this run: --subs, where 'auto' is north_star's MTU 9000 half and
    BASELINE config 3 at N=1, and config 4 (spread landing) at N>1.  Only beside an
    own-landing headline."""
    if args.landing != "own":
        return []
    if args.subs == "auto":
        return ["mtu9000", "config3"] if world == 1 else ["spread"]
    return [s for s in args.subs.split(",") if s and s != "none"]


class Env:
    def __init__(self, **kw):
        self.__dict__.update(kw)


# sub-legs of the driver's default run (--subs): north_star's MTU 9000 half at 1 MiB, and
# BASELINE config 3 (8 MiB events at MTU 9000, 70 events = 65,730 datagrams per launch)
SUB_LEGS = {
    "mtu9000": {"mtu": 9000},
    "config3": {"mtu": 9000, "event_bytes": 8 << 20, "events": 280, "batch_events": 70},
    "spread": {"landing": "spread"},
}


def run_workload(args, env, headline: bool):
    """One workload: inputs resident in HBM, warmup, a byte-exact round-trip check, the
    timed steps (max over ranks), per-kernel HIP-event durations and the roofline.
    Returns the JSON line (without cpu_baseline)."""
    torch, dist, sar, ctx, dev = env.torch, env.dist, env.sar, env.ctx, env.dev
    world, rank, backend, coll_dev = env.world, env.rank, env.backend, env.coll_dev
    B = args.event_bytes
    E = args.events
    seg = sar.DeviceSegmenter(ctx, mtu=args.mtu, lb_hdr_version=args.lb_version)
    mp, stride = seg.max_pld, seg.stride
    npk = sar.num_packets(B, mp)
    G = graph_steps(args)

    # ---- inputs resident in HBM: event bytes + per-batch descriptor tables ----
    ev_stride = (B + 255) // 256 * 256

    def make_src(r):
        """Rank r's source events (regenerable from its seed by any rank, for verification)."""
        g = torch.Generator(device=dev)
        g.manual_seed(0xE25A2 + r)
        s = torch.randint(0, 256, (E, ev_stride), dtype=torch.uint8, device=dev, generator=g)
        if args.payload == "perf":
            head, tail = b"This is a start of event payload", b"...the end"
            assert B >= len(head) + len(tail)
            s.zero_()
            s[:, :len(head)] = torch.tensor(list(head), dtype=torch.uint8, device=dev)
            s[:, B - len(tail):B] = torch.tensor(list(tail), dtype=torch.uint8, device=dev)
        return s

    src = make_src(rank)
    if args.landing == "own":
        evnum = lambda i: i * world + rank      # every local event is owned here: eventNum % world == rank
    else:
        evnum = lambda i: rank * E + i          # owners spread over all ranks: datagrams must be exchanged
    def make_plans(batch):
        out = []
        for b0 in range(0, E, batch):
            idx = range(b0, min(E, b0 + batch))
            out.append(seg.plan([(src[i].data_ptr(), B, evnum(i), 4321, 1 + (evnum(i) * 0x9E37) % 65535,
                                  (1 << 48) + evnum(i)) for i in idx]))
        return out

    plans = make_plans(args.batch_events)
    groups = [seg.groups(p) for p in plans] if args.xcd_groups else None
    if args.guided:
        # A/B: guided group sizes for the fused kernel (e2sar_hip_reassemble_groups with a
        # host-built table): group k takes ceil(remaining / (F x resident)) datagrams, clamped
        # to [SMIN, 64], so the groups dispatched last are the smallest and the launch's
        # workgroups finish together
        # optional 4th/5th values LO,HI: the first RESIDENT groups take sizes spread over
        # [LO, HI] (golden-ratio sequence), so the first residency wave does not finish -- and
        # the second does not classify -- all at once
        vals = [float(x) for x in args.guided.split(",")]
        f, smin, resident = vals[:3]
        lo_hi = vals[3:5] if len(vals) >= 5 else None
        groups = []
        for p in plans:
            st, cur, n_, k = [0], 0, p.total_packets, 0
            while cur < n_:
                if lo_hi and k < resident:
                    fr = (k * 0.6180339887) % 1.0
                    sz = int(round(lo_hi[0] + (lo_hi[1] - lo_hi[0]) * fr))
                else:
                    sz = -(-(n_ - cur) // int(f * resident))
                sz = int(min(64, max(smin, sz)))
                cur = min(n_, cur + sz)
                st.append(cur)
                k += 1
            groups.append((torch.tensor(st, dtype=torch.int32, device=dev), len(st) - 1))
    max_batch_pk = max(p.total_packets for p in plans)
    step_pk = sum(p.total_packets for p in plans)
    if args.reas in ("pipelined", "chained") and args.overlap:
        args.overlap = False                    # the pipeline is its own overlap
    nbuf = 2 if (args.overlap or args.reas == "pipelined") else 1
    if args.lanes > 1:
        if args.overlap or args.reas != "fused" or args.landing != "own":
            raise SystemExit("--lanes runs the fused own-landing step")
        nbuf = args.lanes
    if args.reas == "chained":
        args.chain_batches = max(1, min(8, args.chain_batches))
        nbuf = min(args.chain_batches, len(plans))
    table = 1
    while table < args.table_factor * E:
        table <<= 1
    from e2sar_amd import _capi
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=max(table, 64), queue_capacity=E + 64,
                              lost_capacity=1024, arena_bytes=E * ev_stride + 4096,
                              flags=_capi.REAS_REFERENCE_ORDER if args.reference_order else 0,
                              group_size=args.reas_group)
    if args.landing == "spread":
        R.set_owner(world, rank)          # reassemble only this rank's events (eventNum % world)
    if args.reference_order and args.reas != "fused":
        raise SystemExit("--reference-order runs through reassemble_batch (--reas fused)")

    spread = args.landing == "spread"
    if spread:
        # BASELINE config 4, per landed batch (e2sar_amd.dist.SpreadPipeline): each batch lands
        # in one reused buffer (as the own-landing leg's); while it is still in the Infinity
        # Cache the datagrams this rank owns are reassembled where they landed (the
        # reassembler is set to this rank's ownership) and the FOREIGN ones are appended to
        # per-owner regions (e2sar_hip_route_append); then batch b's counts are all-gathered
        # and its regions exchanged (RCCL all-to-all over xGMI) on a communication stream and
        # what arrived is reassembled (classify + scatter, streaming loads) on a third stream,
        # while batch b+1 lands: the step costs max(landing, exchange), not their sum
        from e2sar_amd.dist import SpreadPipeline
        land = seg.alloc_packets(max_batch_pk)
        pipe = SpreadPipeline(ctx, R, stride, max_batch_pk, world, rank)
        R.set_cold(True)                   # received datagrams: streaming loads in the scatter
        if args.overlap or not args.eager or args.reas != "fused":
            log(args, "landing=spread: per-batch exchange reads split sizes on the host -> eager, fused, no overlap")
        args.overlap = False
        args.reas = "fused"
        args.eager = True
        bufs = []
    else:
        bufs = [seg.alloc_packets(max_batch_pk) for _ in range(nbuf)]
    works = [R.alloc_work(max_batch_pk) for _ in range(nbuf)] if args.reas in ("split", "pipelined") else None
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

    def timed_on(name, stream, fn, *a, **kw):
        """timed() for a launch on an explicit stream (the spread pipeline's three streams)."""
        if not timing_on[0]:
            return fn(*a, stream=stream, **kw)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r = fn(*a, stream=stream, **kw)
        e1.record(stream)
        timing.append((name, e0, e1))
        return r

    if spread:
        pipe.timed = timed_on

    # reassemble_batch runs classify + scatter inside for batches above 320 MiB of slots
    # (e2sar_hip.h); the timing entry then covers both launches
    fused_name = ("reassemble_batch_ro" if args.reference_order else
                  "reas_kernel" if max_batch_pk * stride <= (320 << 20) else "reassemble_batch_split")

    def reassemble(pk, ln, n, k, stream=None):
        """The receive side of one batch: one fused launch, or classify + scatter."""
        if args.reas == "fused" and groups is not None and groups[k][1]:
            timed(fused_name, R.reassemble_groups, pk, stride, ln, n, groups[k][0], groups[k][1], stream=stream)
        elif args.reas == "fused":
            timed(fused_name, R.reassemble, pk, stride, ln, n, stream=stream)
        else:
            w = works[k % nbuf]
            timed("reas_classify_kernel", R.classify, pk, stride, ln, n, w, stream=stream)
            timed("reas_scatter_kernel", R.scatter, pk, stride, n, w, stream=stream)

    def step_spread():
        """Datagrams land on this rank whatever their owner (SpreadPipeline): this rank's
        events are reassembled in place (hot), the foreign ones routed per batch, exchanged
        (RCCL all-to-all) and reassembled by their owners while the next batch lands."""
        lpk, lln = land
        R.recycle(force=True)
        pipe.begin_step()
        for p in plans:
            timed("seg_kernel", seg.segment, p, lpk, lln)
            pipe.land(lpk, lln, p.total_packets)
        pipe.flush()

    def step():
        """One step: recycle the event table/arena, then segment -> reassemble every batch.
        With --overlap, reassembly of batch b runs on a second stream concurrently with
        segmentation of batch b+1 (double-buffered datagram slots)."""
        s0 = torch.cuda.current_stream()
        if spread:
            return step_spread()
        # the default step recycles in its first segmentation launch (extra workgroups at the
        # end of seg_kernel's grid, e2sar_hip_segment_batch_recycle): one launch fewer per step
        fold = args.fold_recycle and args.reas in ("fused", "split") and not args.overlap and args.lanes == 1
        if not fold:
            R.recycle(force=True)
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
        if args.reas == "chained":
            K = args.chain_batches
            for c0 in range(0, len(plans), K):
                chunk = plans[c0:c0 + K]
                timed("segreas_kernel", seg.segment_reassemble_batches, chunk,
                      [bufs[(c0 + j) % nbuf] for j in range(len(chunk))], R)
            return
        if args.lanes > 1 and not timing_on[0]:
            for ls in lane_streams:
                ls.wait_stream(s0)
            for k, p in enumerate(plans):
                ls = lane_streams[k % args.lanes]
                pk, ln = bufs[k % args.lanes]
                seg.segment(p, pk, ln, stream=ls)
                R.reassemble(pk, stride, ln, p.total_packets, stream=ls)
            for ls in lane_streams:
                s0.wait_stream(ls)
            return
        if not args.overlap:
            for k, p in enumerate(plans):
                pk, ln = bufs[k % nbuf] if args.lanes > 1 else bufs[0]
                if k == 0 and fold:
                    timed("seg_kernel", seg.segment, p, pk, ln, recycle=R, force=True)
                else:
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
    lane_streams = [torch.cuda.Stream() for _ in range(args.lanes)] if args.lanes > 1 else []

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # ---- correctness gate (outside the timed region): every event byte-exact ----
    def verify_spread():
        recs = R.poll()
        st = R.stats()
        arena = R.arena_tensor()
        owned = sum(1 for r in range(world) for i in range(E) if (r * E + i) % world == rank)
        ok = (len(recs) == owned and st.inProgress == 0 and st.badHeaderDiscards == 0 and st.dataErrCnt == 0
              and all(r.numFragments == npk for r in recs))
        by_src = {}
        for r in recs:
            by_src.setdefault(r.eventNum // E, []).append(r)
        for s_rank, rs in sorted(by_src.items()):
            if not ok:
                break
            s = src if s_rank == rank else make_src(s_rank)
            for r in rs:
                if not torch.equal(arena[r.arenaOffset: r.arenaOffset + B], s[r.eventNum % E, :B]):
                    ok = False
                    break
            del s
        if not ok:
            raise SystemExit(f"rank {rank}: spread-landing verification FAILED ({len(recs)} records, "
                             f"{owned} owned)")
        return True

    def verify():
        if spread:
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

    def capture(fn, steps):
        """`steps` calls of fn as one HIP graph (kills per-launch host overhead)."""
        graph = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream()
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            fn()                            # warm the capture stream once
        torch.cuda.synchronize()
        with torch.cuda.graph(graph, stream=cap):
            for _ in range(steps):
                fn()
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        return graph

    graph = None
    if not args.eager:
        graph = capture(step, G)
        if not args.no_verify:
            verified = verify() and verified is not False

    def run_timed(fn, g, k, gs=None):
        """k steps (k/G graph replays, or k eager steps) between barriers; max over ranks.
        With --warm-timed (default), the warmup steps are replayed once more right before the
        barrier, the same way the timed steps run, so the timed region starts with the GPU in
        the state the steps keep it in rather than after the verification's host work."""
        if args.warm_timed and args.warmup > 0:
            if g is not None:
                for _ in range(-(-args.warmup // (gs or G))):
                    g.replay()
            else:
                for _ in range(args.warmup):
                    fn()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if g is not None:
            for _ in range(k // (gs or G)):
                g.replay()
        else:
            for _ in range(k):
                fn()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if world > 1:
            dist.barrier()
        el = t1 - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # ---- timed region ----
    K = args.steps
    elapsed = run_timed(step, graph, K)
    # ...and the events the timed steps left behind, byte for byte (outside the timed region)
    if not args.no_verify:
        verified = verify() and verified is not False

    # ---- per-kernel durations: HIP events around each launch of the step, eager, on the
    # stream the kernels run on (the step is single-stream unless --overlap) ----
    def kernel_times(fn, steps):
        timing.clear()
        timing_on[0] = True
        if not spread:
            # keep the GPU behind the host for the whole pass: a spin kernel in front lets
            # every launch and event pair be queued before the GPU reaches them, so a pair
            # brackets GPU time only.  Without it, short eager launches (the cold leg's
            # classify, recycle) drain the queue and the host's launch overhead for the next
            # launch lands inside that launch's event pair: cold leg 82.3 us per launch by
            # events against 78.5 us by rocprof, classify 23.3 against 12.4 (round 5).
            torch.cuda._sleep(int(20e6) * max(1, steps))
        for _ in range(max(1, steps)):
            fn()
        torch.cuda.synchronize()
        timing_on[0] = False
        per = {}
        for name, e0, e1 in timing:
            per.setdefault(name, []).append(e0.elapsed_time(e1))
        return per

    was_overlap = args.overlap
    args.overlap = False
    per = kernel_times(step, args.roofline_steps)
    args.overlap = was_overlap
    avg = {k: sum(v) / len(v) for k, v in per.items()}
    per_launch_events = sum(p.n_events for p in plans) / len(plans)
    # algorithmic bytes of one launch of each bandwidth kernel:
    #   seg: B + (B + 36N) per event; reassembly (fused, scatter, scatter+classify): (B + 36N) + B
    #   (the classify share of scatter+classify -- 24 B of header/length read and 16 B of
    #   record written per datagram -- is left out, so its rate is understated by ~1 %)
    launch_bytes = per_launch_events * (2 * B + 36 * npk)
    bw_kernels = [k for k in avg if k in ("seg_kernel", "reas_kernel", "reas_scatter_kernel",
                                          "reas_scatter_classify_kernel", "segreas_kernel",
                                          "reassemble_batch_split", "reassemble_batch_ro")]
    dom = max(bw_kernels, key=lambda k: sum(per[k]))      # most time in the step
    dom_ms = avg[dom]
    if spread and dom == "reas_kernel":
        # the in-place launches reassemble the events that landed here AND are owned here
        # (eventNum = rank * E + i): their payload, plus every landed datagram's 36-byte
        # header read to find out (the foreign payloads are not loaded)
        here = sum(1 for i in range(E) if (rank * E + i) % world == rank)
        launch_bytes = (here * (2 * B) + E * 36 * npk) / len(plans)
    if dom == "segreas_kernel":
        launch_bytes *= 2                       # both stages' bytes in one launch: 4B + 72N per event
    achieved = launch_bytes / (dom_ms * 1e-3) / 1e9

    # HBM traffic per launch of the dominant kernel, from the committed rocprofv3 PMC passes
    # of this same workload (tools/pmc_summary.py; FETCH_SIZE x2 + WRITE_SIZE, gfx950 rules)
    traffic, traffic_src = (None, None) if (spread or args.reas != "fused" or args.overlap) else _pmc_traffic(args, dom)

    # achievable HBM on this device beside the 8 TB/s peak: a plain copy of this
    # rank's source events (1 GiB) into the arena with e2sar_hip_copy_spans (16-byte
    # non-temporal loads and stores, one 16-KiB piece per workgroup), HIP events around 5 copies
    copy_gbps, copy_per = None, None
    if headline and not spread:
        copy_gbps, copy_per = copy_calibration(ctx, torch, dev)

    # spread landing: the exchange's bytes against the xGMI links: this rank's
    # datagram slots + lengths sent to other ranks per step / the exchange's time
    xgmi = None
    if spread and world > 1 and "exchange" in per and sum(per["exchange"]) > 0:
        # per step: this rank's foreign datagram slots + lengths sent / the exchanges' time
        # (the step's all-to-alls, each timed on the communication stream; they overlap the
        # landing of the next batch, so their sum is not a share of the step)
        sent = pipe.sent * (stride + 4)
        ex_ms = sum(per["exchange"]) / max(1, args.roofline_steps)
        xgmi = {"bytes_sent_per_step": sent, "exchange_ms_per_step": round(ex_ms, 5),
                "exchanges_per_step": len(per["exchange"]) // max(1, args.roofline_steps),
                "achieved": round(sent / (ex_ms * 1e-3) / 1e9, 1), "peak": XGMI_PEAK_GBS,
                "unit": "GB/s", "frac": round(sent / (ex_ms * 1e-3) / 1e9 / XGMI_PEAK_GBS, 4),
                "backend": backend}

    total_payload = E * B * world * K
    value = total_payload / elapsed / 2**30
    step_bytes = E * (4 * B + 72 * npk)

    # ---- cold receive-only leg: every batch's datagrams in a buffer of its own, written
    # once before timing; a step reassembles them all (1.1 GB of datagrams > the 256 MiB
    # Infinity Cache, so each launch reads its batch back from HBM) ----
    cold = None
    if args.cold_steps > 0 and not spread:
        # a reassembler of its own, told its datagrams are cold (streaming loads in the
        # scatter, E2SAR_HIP_REAS_COLD_DATAGRAMS); verify() and the steps below use it
        R_hot = R
        R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=max(table, 64), queue_capacity=E + 64,
                                  lost_capacity=1024, arena_bytes=E * ev_stride + 4096,
                                  flags=_capi.REAS_COLD_DATAGRAMS)
        cb = args.cold_batch_events or E
        cplans = plans if cb == args.batch_events else make_plans(cb)
        cbufs = [seg.alloc_packets(p.total_packets) for p in cplans]
        for p, (pk, ln) in zip(cplans, cbufs):
            seg.segment(p, pk, ln)
        cmax_pk = max(p.total_packets for p in cplans)
        cwork = [R.alloc_work(cmax_pk) for _ in range(2)] if args.cold_reas != "fused" else None
        torch.cuda.synchronize()

        def cstep():
            R.recycle(force=True)
            if args.cold_reas == "pipelined":
                p0, (pk0, ln0) = cplans[0], cbufs[0]
                timed("reas_classify_kernel", R.classify, pk0, stride, ln0, p0.total_packets, cwork[0])
                for k, (p, (pk, ln)) in enumerate(zip(cplans, cbufs)):
                    if k + 1 < len(cplans):
                        q, (qpk, qln) = cplans[k + 1], cbufs[k + 1]
                        timed("reas_scatter_classify_kernel", R.scatter_classify, stride, pk, p.total_packets,
                              cwork[k % 2], qpk, qln, q.total_packets, cwork[(k + 1) % 2])
                    else:
                        timed("reas_scatter_kernel", R.scatter, pk, stride, p.total_packets, cwork[k % 2])
                return
            for p, (pk, ln) in zip(cplans, cbufs):
                if cwork is None:
                    timed("reas_kernel", R.reassemble, pk, stride, ln, p.total_packets)
                else:
                    timed("reas_classify_kernel", R.classify, pk, stride, ln, p.total_packets, cwork[0])
                    timed("reas_scatter_kernel", R.scatter, pk, stride, p.total_packets, cwork[0])

        cstep()
        torch.cuda.synchronize()
        cver = None if args.no_verify else verify()
        # the cold leg's own graph: all its --cold-steps in one graph (up to 64), as the step's
        Gc = args.graph_steps or next(d for d in range(min(args.cold_steps, 64), 0, -1) if args.cold_steps % d == 0)
        cgraph = None if args.eager else capture(cstep, Gc)
        ck = max(Gc, args.cold_steps // Gc * Gc)
        cel = run_timed(cstep, cgraph, ck, Gc)
        cper = kernel_times(cstep, args.roofline_steps)
        ckern = {"fused": "reas_kernel", "split": "reas_scatter_kernel",
                 "pipelined": "reas_scatter_classify_kernel"}[args.cold_reas]
        if ckern not in cper:                   # pipelined form with one batch: classify + scatter
            ckern = "reas_scatter_kernel"
        c_ms = sum(cper[ckern]) / len(cper[ckern])
        # per launch of ckern: the batches it scatters (the last batch's scatter-only launch
        # is not ckern in the pipelined form)
        c_ev = [p.n_events for p in cplans]
        c_ev = c_ev[:-1] if ckern == "reas_scatter_classify_kernel" else c_ev
        c_bytes = sum(c_ev) / len(c_ev) * (2 * B + 36 * npk)
        c_ach = c_bytes / (c_ms * 1e-3) / 1e9
        cold = {
            "what": f"reassembly alone ({args.cold_reas} form) on datagrams written long before (one buffer "
                    f"per batch, {step_pk * stride / 1e9:.2f} GB per step, read back from HBM); value = payload "
                    "reassembled per second",
            "batch_events": cb,
            "form": {"fused": "reas_kernel per batch",
                     "split": "reas_classify_kernel + reas_scatter_kernel per batch",
                     "pipelined": "reas_classify_kernel(0), then reas_scatter_classify_kernel: scatter(b) "
                                  "beside classify(b+1)"}[args.cold_reas],
            "value": round(E * B * world * ck / cel / 2**30, 3), "unit": "GiB/s", "steps": ck,
            # the whole leg (every launch: classify, scatter, recycle) against the same peak
            "leg_achieved_GBps": round(E * (2 * B + 36 * npk) * ck / cel / 1e9, 1),
            "leg_frac": round(E * (2 * B + 36 * npk) * ck / cel / 1e9 / HBM_PEAK_GBS, 4),
            "ms_per_step": round(cel / ck * 1e3, 4), "verified": cver,
            "roofline": {"bound": "hbm", "kernel": ckern, "achieved": round(c_ach, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(c_ach / HBM_PEAK_GBS, 4),
                         "avg_launch_ms": round(c_ms, 5), "algorithmic_bytes_per_launch": int(c_bytes),
                         "all_launch_ms": {k: round(sum(v) / len(v), 5) for k, v in cper.items()}},
            "flags": "E2SAR_HIP_REAS_COLD_DATAGRAMS",
        }
        ctr, csrc = _pmc_traffic(args, ckern, batch_events=cb)
        cold["roofline"]["traffic"] = ctr
        if ctr is not None:
            cold["roofline"]["traffic_unit"] = "bytes per launch (rocprofv3 PMC, committed)"
            cold["roofline"]["traffic_source"] = csrc
        del cbufs
        R.close()
        R = R_hot

    if True:
        line = {
            "metric": METRIC,
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
                "parallelism": (f"eventNum % {world} sharding (no collective)" if not spread else
                                f"eventNum % {world} owners, datagrams land spread: route + all-to-all-v "
                                f"({backend}) + reassemble"),
                "launch": ("eager, three streams: landing (segment, in-place reassembly, route) | count "
                           "all-gather + all-to-all | reassembly of what arrived" if spread and world > 1 else
                           "eager" if args.eager else f"hipGraph of {G} step(s), replayed {K // G} times"),
                "overlap": bool(args.overlap),
                "lanes": args.lanes,
                "xcd_groups": bool(groups and all(g[1] for g in groups)),
                "reassembly": {"fused": ("reas_kernel per batch" if fused_name == "reas_kernel" else
                                         "reassemble_batch per batch, REFERENCE_ORDER: key pass (runs filed "
                                         "per key), per-key walk, scatter" if args.reference_order else
                                         "reassemble_batch per batch: classify + scatter launches inside "
                                         "(batch above 320 MiB of slots)"),
                               "split": "reas_classify_kernel + reas_scatter_kernel per batch",
                               "pipelined": "reas_scatter_classify_kernel: scatter(b) beside classify(b+1), "
                                            "2 datagram buffers",
                               "chained": "segreas_kernel per batch: seg blocks then reassembly groups in one "
                                          "launch, per-group ready counters"}[args.reas],
                "landing": args.landing,
                "payload": args.payload,
                "verified_roundtrip": verified,
                "verified_at": None if args.no_verify else
                ["an eager step", "the captured graph's first replay", "the timed steps' last step"]
                if graph is not None else ["an eager step", "the timed steps' last step"],
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
                "copy_GBps": round(copy_gbps, 1) if copy_gbps else None,
                "copy_what": ("best device-to-device copy on this GPU (e2sar_hip_copy_spans, 16-B non-temporal "
                              "loads/stores, 8-KiB pieces) of 1 and 4 GiB of random bytes, read + write bytes"),
                "copy_GBps_by_size": copy_per,
                "frac_of_copy": round(achieved / copy_gbps, 4) if copy_gbps else None,
                # the best plain copy ever measured on MI355X in this repository (DESIGN 4.3:
                # tools/ubench_copy.hip, aligned 16-B non-temporal copy of 1 GiB), so the
                # fraction is never taken against a slower copy than the best one known
                "best_copy_GBps": BEST_COPY_GBS,
                "frac_of_best_copy": round(achieved / max(BEST_COPY_GBS, copy_gbps or 0.0), 4),
            },
            "xgmi": xgmi,
            "reas_cold": cold,
        }
        if spread:
            line["spread"] = {"foreign_sent_per_step": pipe.sent, "received_per_step": pipe.received,
                              "route": "foreign only, per batch (e2sar_hip_route_append into per-owner regions)",
                              "in_place": "reas_kernel with e2sar_hip_reas_set_owner(world, rank)",
                              "exchange": "per batch: count all-gather + all_to_all on a communication stream, "
                                          "overlapping the next batch's landing (dist.SpreadPipeline)",
                              "received_form": "reas_classify + reas_scatter (streaming loads) on a third stream"}
    # free this workload's device buffers before the next one (sub-legs)
    R.close()
    return line

if __name__ == "__main__":
    main()
