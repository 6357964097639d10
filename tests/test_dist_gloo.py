"""N>1 path on CPU: world_size 2 over gloo.

Datagrams of 8 events land on the two ranks by packet index (a modelled NIC spread), so
every event has fragments on both ranks.  Each rank routes its landed batch by owner
(eventNum % world) with the same stable packing the gfx950 route kernels implement,
exchanges spans with e2sar_amd.dist.exchange (all_to_all_single), and reassembles what
it received with the oracle: every rank must end with exactly the events it owns, whole.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def stable_route(pk, ln, world, self_rank, with_lb=True):
    """Host restatement of route_hist/scan/pack (test helper): stable per-owner spans."""
    import oracle_ffi as O
    hl = 36 if with_lb else 20
    dests = []
    for k in range(len(ln)):
        okv, _, _, _, ev, _ = O.re_parse(pk[k, (16 if with_lb else 0):].tobytes()) if ln[k] >= hl else (False,) * 6
        dests.append(int(ev) % world if okv else self_rank)
    order = [k for d in range(world) for k in range(len(ln)) if dests[k] == d]
    counts = [sum(1 for x in dests if x == d) for d in range(world)]
    return pk[order], ln[order], counts


def _worker(rank, world, port, result_q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import oracle_ffi as O
    import sar_inputs as S
    from e2sar_amd.dist import exchange, owner

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        mp_ = O.max_pld_len(1500)
        stride = (36 + mp_ + 15) // 16 * 16
        evs = [S.event_bytes(i, 5000 + 311 * i) for i in range(8)]
        pks, lns = [], []
        for i, e in enumerate(evs):
            p, l = O.segment_event(e, i, S.DATA_ID, S.entropy(i), S.lb_tick(i), 2, mp_, stride)
            pks.append(p)
            lns.append(l)
        allp = np.concatenate(pks)
        alll = np.concatenate(lns)
        landed = np.arange(len(alll)) % world == rank
        spk, sln, counts = stable_route(allp[landed], alll[landed], world, rank)
        rpk, rln, n = exchange(torch.from_numpy(spk.reshape(-1).copy()),
                               torch.from_numpy(sln.astype(np.int32)), counts, stride)
        rpk = rpk[: n * stride].numpy().reshape(n, stride)
        rln = rln[:n].numpy().astype(np.uint32)
        # the oracle needs each event's offset-0 fragment first (cpp:361-369); the spans
        # arrive grouped by source rank, so feed it in (eventNum, offset) order
        key = [(int.from_bytes(rpk[k, 28:36].tobytes(), "big"), int.from_bytes(rpk[k, 20:24].tobytes(), "big"))
               for k in range(n)]
        order = sorted(range(n), key=lambda k: key[k])
        r = O.Reassembler(True)
        r.push_batch(rpk[order], rln[order])
        got = {e: b for b, e, d in r.pop_all()}
        mine = [i for i in range(8) if owner(i, world) == rank]
        ok = sorted(got) == mine and all(got[i] == evs[i].tobytes() for i in mine)
        st = r.stats()
        ok = ok and st["inProgress"] == 0 and st["badHeaderDiscards"] == 0
        result_q.put((rank, ok, sorted(got), n))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2])
def test_exchange_then_reassemble_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    res = sorted(q.get(timeout=5) for _ in range(world))
    for rank, ok, got, n in res:
        assert ok, (rank, got, n)
        assert got == [i for i in range(8) if i % world == rank]
    assert all(p.exitcode == 0 for p in procs)


def test_stable_route_matches_owner_rule():
    import oracle_ffi as O
    mp_ = O.max_pld_len(1500)
    pk, ln = O.segment_event(np.arange(4000, dtype=np.uint8), 5, 1, 2, 3, 2, mp_, 1472)
    spk, sln, counts = stable_route(pk, ln, 4, 0)
    assert counts == [0, len(ln), 0, 0]
    bad = pk.copy()
    bad[0, 16] = 0x20
    _, _, counts = stable_route(bad, ln, 4, 3)
    assert counts == [0, len(ln) - 1, 0, 1]
