"""Config 4 on the HIP path: datagrams land spread over the ranks, the owner of an event is
eventNum % world, and every rank must end with exactly the events it owns.

Two forms of the receive side are checked, each rank's events and counters against the
oracle's reassembly of the datagrams that rank processed:

* ``all``: route every landed datagram to its owner (e2sar_hip_route_batch, self
  included), one all-to-all-v, reassemble what arrived;
* ``foreign``: reassemble the datagrams this rank owns where they landed
  (e2sar_hip_reas_set_owner), route only the foreign ones (e2sar_hip_route_foreign),
  exchange them (split sizes from one all-gather of the device count vectors), reassemble
  what arrived;
* ``regions``: as ``foreign``, but the landed stream comes in batches, each routed into
  per-rank regions right after it landed (e2sar_hip_route_append), and one exchange of the
  regions follows the last batch;
* ``pipeline`` (what bench.py's spread sub-leg runs, dist.SpreadPipeline): per batch,
  in-place reassembly, routing, then that batch's exchange and the reassembly of what it
  brought (on their own streams with RCCL); ``pipeline_all`` routes every datagram through
  the exchange.

Two ranks share GPU 0 over gloo (all-to-all staged through host memory; RCCL refuses two
ranks on one device).  The RCCL branch itself runs at world 1 in a fresh child process
that initialises the ``nccl`` process group before any other GPU call: route -> exchange
(device tensors through RCCL) -> reas_kernel, in both forms, against the oracle.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _spread_rank(rank, world, mode, corrupt=True):
    """One rank's share of the spread-landing case; returns the fields the parent checks."""
    import torch

    import oracle_ffi as O
    import sar_inputs as S
    from e2sar_amd import sar
    from e2sar_amd.dist import PacketRouter, RegionRouter, exchange

    ctx = sar.Context(0)
    mtu = 1500
    sizes = [5000 + 7919 * i for i in range(10)] + [1, 1436, 1437]
    evs = [S.event_bytes(100 + i, s) for i, s in enumerate(sizes)]
    seg = sar.DeviceSegmenter(ctx, mtu=mtu, lb_hdr_version=2)
    stride = seg.stride
    # every rank segments the same events (deterministic); datagram k of the stream
    # "lands" on rank k % world (a modelled NIC spread), so every multi-datagram event
    # has fragments on every rank
    offs, cur = [], 0
    for e in evs:
        cur = (cur + 255) // 256 * 256
        offs.append(cur)
        cur += len(e)
    host = np.zeros(cur, np.uint8)
    for e, o in zip(evs, offs):
        host[o:o + len(e)] = e
    dsrc = torch.from_numpy(host).to(ctx.torch_device)
    plan = seg.plan([(dsrc.data_ptr() + o, len(e), 100 + i, S.DATA_ID, S.entropy(i), S.lb_tick(i))
                     for i, (e, o) in enumerate(zip(evs, offs))])
    pk, ln = seg.alloc_packets(plan.total_packets)
    seg.segment(plan, pk, ln)
    n = plan.total_packets
    landed = torch.arange(n, device=ctx.torch_device) % world == rank
    lpk = pk[: n * stride].view(n, stride)[landed].contiguous().view(-1)
    lln = ln[:n][landed].contiguous()
    nl = int(landed.sum())
    if corrupt and rank == world - 1:
        lpk[16] = 0x20                    # RE version 2: unparsable, stays on the landing rank
    router = PacketRouter(ctx, stride, nl, world, rank)
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=256, arena_bytes=1 << 22)
    hp_l = lpk[: nl * stride].view(nl, stride).cpu().numpy()
    hl_l = lln[:nl].cpu().numpy().astype(np.uint32)
    if mode in ("pipeline", "pipeline_all"):
        # dist.SpreadPipeline (bench.py's spread sub-leg): landed batches, each reassembled in
        # place and routed, its exchange and the reassembly of
        # what it brought on their own streams (RCCL) or synchronous (gloo); pipeline_all
        # routes every datagram, own included, through the exchange
        from e2sar_amd.dist import SpreadPipeline
        in_place = mode == "pipeline"
        if in_place:
            R.set_owner(world, rank)
        pipe = SpreadPipeline(ctx, R, stride, nl, world, rank, in_place=in_place)
        R.set_cold(True)
        # what each exchange brought, copied on the stream that reassembles it (the receive
        # sets rotate, so a later batch overwrites them)
        arrived = []
        reas_rx = pipe._reassemble_received

        def keep_copy(rpk_, rln_, n_, work_, stream_):
            with torch.cuda.stream(stream_ if stream_ is not None else torch.cuda.current_stream()):
                arrived.append((rpk_[: n_ * stride].clone(), rln_[:n_].clone()))
            reas_rx(rpk_, rln_, n_, work_, stream_)

        pipe._reassemble_received = keep_copy
        pipe.begin_step()
        # five batches (cuts inside events): with the default depth 3 the exchanges of the
        # first three are issued by later land() calls and region / receive sets are reused
        cuts = [0] + [nl * k // 5 + k for k in range(1, 5)] + [nl]
        for a, b in zip(cuts[:-1], cuts[1:]):
            if b > a:
                pipe.land(lpk[a * stride:], lln[a:], b - a)
        pipe.flush()
        torch.cuda.synchronize()
        nr = sum(c for _, c in pipe.recv_log)
        assert nr == sum(x[1].numel() for x in arrived)
        rpk = torch.cat([x[0] for x in arrived] + [lpk[:0]])
        rln = torch.cat([x[1] for x in arrived] + [lln[:0]])
        counts = [sum(m[rank][d] for m in pipe.matrices) for d in range(world)]
        keep = []
        for k in range(nl):
            ok, _, _, _, e, _ = O.re_parse(hp_l[k, 16:36].tobytes())
            parsable = ok and 36 <= hl_l[k] <= stride
            keep.append(in_place and (not parsable or e % world == rank))
        keep = np.array(keep, bool)
    elif mode in ("foreign", "regions"):
        R.set_owner(world, rank)
        if mode == "foreign":
            R.reassemble(lpk, stride, lln, nl)                # this rank's events, in place
            spk, sln, cnt = router.route(lpk, lln, nl, foreign_only=True)
            rpk, rln, nr = exchange(spk, sln, cnt, stride)   # device counts: one host read
            counts = [int(c) for c in cnt.tolist()]
        else:
            # bench.py's spread leg: the landed stream in batches (a cut inside events), each
            # reassembled in place and appended to per-rank regions, one exchange at the end
            rr = RegionRouter(ctx, stride, nl, nl, world, rank)
            rr.reset()
            cut = nl // 3 + 1
            for a, b in ((0, cut), (cut, nl)):
                R.reassemble(lpk[a * stride:], stride, lln[a:], b - a)
                rr.route(lpk[a * stride:], lln[a:], b - a)
            rpk, rln, nr = rr.exchange()
            counts = [int(c) for c in rr.running.tolist()]
        R.set_cold(True)
        R.reassemble(rpk, stride, rln, nr)
        # what this rank processed: the landed datagrams it keeps + what it received
        keep = []
        for k in range(nl):
            ok, _, _, _, e, _ = O.re_parse(hp_l[k, 16:36].tobytes())
            parsable = ok and 36 <= hl_l[k] <= stride
            keep.append(not parsable or e % world == rank)
        keep = np.array(keep, bool)
    else:
        spk, sln, cnt = router.route(lpk, lln, nl)
        counts = [int(c) for c in cnt.tolist()]
        rpk, rln, nr = exchange(spk, sln, counts, stride)
        R.reassemble(rpk, stride, rln, nr)
        keep = np.zeros(nl, bool)
    torch.cuda.synchronize()
    got = {(r.eventNum, r.dataId): (R.event_bytes(r), r.numFragments) for r in R.poll()}
    st = R.stats()
    hp_r = rpk[: nr * stride].view(nr, stride).cpu().numpy() if nr else np.zeros((0, stride), np.uint8)
    hl_r = rln[:nr].cpu().numpy().astype(np.uint32) if nr else np.zeros(0, np.uint32)
    hp = np.concatenate([hp_l[keep], hp_r])
    hl = np.concatenate([hl_l[keep], hl_r])
    # oracle over the same datagrams; offset 0 first per event (the device path is
    # order-insensitive, the reference replaces an item on a late offset 0)
    m = len(hl)
    key = [(int.from_bytes(hp[k, 28:36].tobytes(), "big"), int.from_bytes(hp[k, 20:24].tobytes(), "big"))
           for k in range(m)]
    order = sorted(range(m), key=lambda k: key[k])
    ro = O.Reassembler(True)
    if m:
        ro.push_batch(hp[order], hl[order])
    ref = {(e, d): b for b, e, d in ro.pop_all()}
    rst = ro.stats()
    mine = sorted(100 + i for i in range(len(sizes)) if (100 + i) % world == rank)
    # the corrupted datagram is stream index world-1 (second fragment of event 100 at
    # world 2): that event stays in progress on its owner
    broken = {100} if (corrupt and world > 1) else set()
    complete = [e for e in mine if e not in broken]
    ok = sorted(e for e, _ in got) == sorted(e for e, _ in ref) == complete
    ok = ok and all(got[k][0] == ref[k] for k in ref)
    ok = ok and all(ref[(e, S.DATA_ID)] == evs[e - 100].tobytes() for e in complete)
    fields = ("eventSuccess", "totalPackets", "totalBytes", "badHeaderDiscards", "dataErrCnt", "inProgress")
    stat_ok = {f: (int(getattr(st, f)), int(rst[f])) for f in fields}
    ok = ok and all(a == b for a, b in stat_ok.values()) and st.errorFlags == 0
    return rank, ok, complete, counts, nr, stat_ok


def _gloo_worker(rank, world, port, mode, result_q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        result_q.put(_spread_rank(rank, world, mode))
    finally:
        dist.destroy_process_group()


def _nccl_worker(port, result_q):
    """World 1 over RCCL: the process group is initialised (device_id given: eager RCCL
    communicator) before any other GPU call of this fresh process."""
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch
    import torch.distributed as dist
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    out = {}
    try:
        assert dist.get_backend() == "nccl"
        # exchange() with host counts: one all_to_all_single of device tensors through RCCL
        from e2sar_amd.dist import exchange
        stride = 64
        n = 1000
        g = torch.Generator(device="cuda")
        g.manual_seed(7)
        spk = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device="cuda", generator=g)
        sln = torch.randint(36, stride + 1, (n,), dtype=torch.int32, device="cuda", generator=g)
        rpk, rln, nr = exchange(spk, sln, [n], stride)
        out["raw"] = bool(nr == n and torch.equal(rpk[: n * stride], spk) and torch.equal(rln[:n], sln)
                          and rpk.is_cuda)
        for mode in ("all", "foreign", "regions", "pipeline", "pipeline_all"):
            out[mode] = _spread_rank(0, 1, mode, corrupt=False)
        # the regions path's RCCL branch (all_to_all over region views) with data in flight:
        # every datagram routed to rank 0 itself (route_append without foreign_only)
        from e2sar_amd.dist import RegionRouter
        from e2sar_amd import sar
        ctx = sar.Context(0)
        rr = RegionRouter(ctx, stride, 2 * n, n, 1, 0, with_lb_header=True, foreign_only=False)
        rr.reset()
        spk2 = spk.clone()
        for k in range(n):                                 # parsable RE headers: version 1, eventNum k
            spk2[k * stride + 16] = 0x10
            spk2[k * stride + 17] = 0
        sln2 = torch.full((n,), stride, dtype=torch.int32, device="cuda")
        rr.route(spk2, sln2, n // 2)
        rr.route(spk2[(n // 2) * stride:], sln2[n // 2:], n - n // 2)
        rpk2, rln2, nr2 = rr.exchange()
        # route_append keeps the order inside each 256-datagram workgroup only (workgroups
        # append in the order they reserve): compare the received slots as a multiset, each
        # slot with its length
        got = torch.cat([rpk2[: n * stride].view(n, stride), rln2[:n].view(n, 1).to(torch.uint8)], 1).cpu()
        want = torch.cat([spk2[: n * stride].view(n, stride), sln2.view(n, 1).to(torch.uint8)], 1).cpu()
        key = lambda t: sorted(bytes(r.numpy()) for r in t)
        out["regions_raw"] = bool(nr2 == n and key(got) == key(want) and torch.equal(rln2[:n], sln2))
        out["backend"] = dist.get_backend()
    finally:
        dist.destroy_process_group()
    result_q.put(out)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(target, args, nproc, timeout=150):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=a + (q,)) for a in args]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(nproc):
            res.append(q.get(timeout=timeout))
    finally:
        for p in procs:
            p.join(timeout=30)
        alive = [p for p in procs if p.is_alive()]
        for p in alive:
            p.kill()
    assert not alive, "rank processes hung"
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return res


@pytest.mark.parametrize("mode", ["all", "foreign", "regions", "pipeline", "pipeline_all"])
def test_spread_landing_route_exchange_reassemble_two_ranks(mode):
    port = _free_port()
    world = 2
    res = sorted(_run(_gloo_worker, [(r, world, port, mode) for r in range(world)], world))
    for rank, ok, mine, counts, nr, stat_ok in res:
        assert ok, (rank, mine, counts, nr, stat_ok)
    # rank 1's unparsable datagram stayed home and was counted there; event 100 (owner rank
    # 0) misses that fragment
    assert res[1][5]["badHeaderDiscards"][0] == 1 and res[0][5]["badHeaderDiscards"][0] == 0
    assert res[0][5]["inProgress"] == (1, 1) and res[1][5]["inProgress"] == (0, 0)
    if mode not in ("all", "pipeline_all"):
        # nothing a rank owns is packed for itself
        assert res[0][3][0] == 0 and res[1][3][1] == 0


def test_rccl_exchange_world1_fresh_process():
    """The nccl (RCCL) branch of dist.exchange on the GPU, route -> exchange -> reassemble."""
    (out,) = _run(_nccl_worker, [(_free_port(),)], 1, timeout=240)
    assert out["backend"] == "nccl"
    assert out["raw"], "RCCL all-to-all of datagram slots changed bytes"
    assert out["regions_raw"], "RCCL all_to_all of region views changed bytes"
    for mode in ("all", "foreign", "regions", "pipeline", "pipeline_all"):
        rank, ok, mine, counts, nr, stat_ok = out[mode]
        assert ok, (mode, mine, counts, nr, stat_ok)
        assert mine == [100 + i for i in range(13)]
    # SpreadPipeline over RCCL: in place nothing moves; routing all, every datagram crosses
    # the count all-gather, the all_to_all and the received-datagram streams
    assert out["pipeline"][3] == [0] and out["pipeline"][4] == 0
    assert out["pipeline_all"][3] == [out["pipeline_all"][4]] and out["pipeline_all"][4] > 0
    # route_batch sends every datagram to rank 0 through RCCL; foreign-only routing keeps them
    assert out["all"][3] == [out["all"][4]] and out["all"][4] > 0
    assert out["foreign"][3] == [0] and out["foreign"][4] == 0
    assert out["regions"][3] == [0] and out["regions"][4] == 0
