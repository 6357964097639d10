"""Config 4 on the HIP path: datagrams land spread over two ranks, are routed to their
owner (eventNum % world) by the gfx950 route kernels, exchanged with
e2sar_amd.dist.exchange, and reassembled by reas_kernel on the owner.

Both ranks share GPU 0 (the one-GPU rehearsal of the 8-GPU node) and talk over gloo, whose
all-to-all stages through host memory; on the node the same code runs over RCCL.  Each
rank's reassembled events and counters must equal the oracle's reassembly of the
datagrams that rank received.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _worker(rank, world, port, result_q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import torch
    import torch.distributed as dist

    import oracle_ffi as O
    import sar_inputs as S
    from e2sar_amd import sar
    from e2sar_amd.dist import PacketRouter, exchange

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ctx = sar.Context(0)
        mtu = 1500
        sizes = [5000 + 7919 * i for i in range(10)] + [1, 1436, 1437]
        evs = [S.event_bytes(100 + i, s) for i, s in enumerate(sizes)]
        seg = sar.DeviceSegmenter(ctx, mtu=mtu, lb_hdr_version=2)
        stride = seg.stride
        # every rank segments the same events (deterministic); datagram k of the stream
        # "lands" on rank k % world (a modelled NIC spread), so every multi-datagram event
        # has fragments on both ranks
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
        if rank == 1:
            lpk[16] = 0x20                    # RE version 2: unparsable, stays on the landing rank
        router = PacketRouter(ctx, stride, nl, world, rank)
        spk, sln, cnt = router.route(lpk, lln, nl)
        counts = [int(c) for c in cnt.tolist()]
        rpk, rln, nr = exchange(spk, sln, counts, stride)
        R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=256, arena_bytes=1 << 22)
        R.reassemble(rpk, stride, rln, nr)
        torch.cuda.synchronize()
        got = {(r.eventNum, r.dataId): (R.event_bytes(r), r.numFragments) for r in R.poll()}
        st = R.stats()
        # oracle over the same received datagrams; offset 0 first per event (the device path
        # is order-insensitive, the reference replaces an item on a late offset 0)
        hp = rpk[: nr * stride].view(nr, stride).cpu().numpy()
        hl = rln[:nr].cpu().numpy().astype(np.uint32)
        key = [(int.from_bytes(hp[k, 28:36].tobytes(), "big"), int.from_bytes(hp[k, 20:24].tobytes(), "big"))
               for k in range(nr)]
        order = sorted(range(nr), key=lambda k: key[k])
        ro = O.Reassembler(True)
        ro.push_batch(hp[order], hl[order])
        ref = {(e, d): b for b, e, d in ro.pop_all()}
        rst = ro.stats()
        mine = sorted(100 + i for i in range(len(sizes)) if (100 + i) % world == rank)
        # the corrupted datagram is stream index 1 = event 100's second fragment: that event
        # (owned by rank 0) stays in progress on both paths
        complete = [e for e in mine if e != 100]
        ok = sorted(e for e, _ in got) == sorted(e for e, _ in ref) == complete
        ok = ok and all(got[k][0] == ref[k] for k in ref)
        ok = ok and all(ref[(e, S.DATA_ID)] == evs[e - 100].tobytes() for e in complete)
        fields = ("eventSuccess", "totalPackets", "totalBytes", "badHeaderDiscards", "dataErrCnt", "inProgress")
        stat_ok = {f: (int(getattr(st, f)), int(rst[f])) for f in fields}
        ok = ok and all(a == b for a, b in stat_ok.values())
        result_q.put((rank, ok, complete, counts, nr, stat_ok))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_spread_landing_route_exchange_reassemble_two_ranks():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "rank processes hung"
    res = sorted(q.get(timeout=5) for _ in range(world))
    for rank, ok, mine, counts, nr, stat_ok in res:
        assert ok, (rank, mine, counts, nr, stat_ok)
    # rank 1's unparsable datagram stayed home and was counted there; event 100 (owner rank
    # 0) misses that fragment
    assert res[1][5]["badHeaderDiscards"][0] == 1 and res[0][5]["badHeaderDiscards"][0] == 0
    assert res[0][5]["inProgress"] == (1, 1) and res[1][5]["inProgress"] == (0, 0)
    assert all(p.exitcode == 0 for p in procs)
