"""dist.SpreadPipeline (BASELINE config 4, bench.py's spread sub-leg) on CPU: world 2 and 3
over gloo, with the GPU pieces replaced by host stand-ins -- a reassembler that records what
it is handed and a region router that packs foreign datagrams by the owner rule
(eventNum % world) as route_append_kernel does.

Per rank: datagrams of 8 events land by packet index (a modelled NIC spread) in 3 batches
cut inside events; every batch is landed through the pipeline (in place + route + the
synchronous gloo exchange).  Every rank must then have been handed exactly the datagrams of
the events it owns -- each once, in place or received -- and nothing else; the count
matrices of every batch must agree across ranks.  The RCCL form (streams, pinned counts,
all_to_all over region views) runs on the GPU: tests/test_gpu_dist.py.
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


class _Ctx:
    torch_device = torch.device("cpu")


def _ev_of(row):
    return int.from_bytes(bytes(row[28:36]), "big")


class _FakeR:
    """Records the datagrams each launch is handed (in place: only this rank's events, as
    a reassembler set to this rank's ownership takes them)."""

    def __init__(self, world, rank, stride):
        self.world, self.rank, self.stride = world, rank, stride
        self.in_place, self.received = [], []

    def _rows(self, pk, ln, n):
        a = pk[: n * self.stride].numpy().reshape(n, self.stride)
        return [(bytes(a[k, : int(ln[k])]), int(ln[k])) for k in range(n)]

    def reassemble(self, pk, stride, ln, n, now_ms=0, stream=None):
        for row, l in self._rows(pk, ln, n):
            if _ev_of(np.frombuffer(row, np.uint8)) % self.world == self.rank:
                self.in_place.append(row)

    def classify(self, pk, stride, ln, n, work, now_ms=0, stream=None):
        self.received += [row for row, _ in self._rows(pk, ln, n)]

    def scatter(self, pk, stride, n, work, stream=None):
        pass

    def alloc_work(self, n):
        return torch.empty(16, dtype=torch.uint8)


class _FakeRouter:
    """route_append_kernel's contract on the host: foreign datagrams appended to region
    d = owner, running[d] counts them (this rank's own stay out with foreign_only)."""

    def __init__(self, ctx, stride, cap, max_batch, world, rank, with_lb_header=True, foreign_only=True):
        self.stride, self.cap, self.world, self.rank, self.foreign_only = stride, cap, world, rank, foreign_only
        self.send_pk = torch.zeros(world * cap * stride, dtype=torch.uint8)
        self.send_ln = torch.zeros(world * cap, dtype=torch.int32)
        self.running = torch.zeros(world, dtype=torch.int32)

    def reset(self, stream=None):
        self.running.zero_()

    def route(self, pk, ln, n, stream=None):
        a = pk[: n * self.stride].view(n, self.stride)
        for k in range(n):
            d = _ev_of(a[k].numpy()) % self.world
            if self.foreign_only and d == self.rank:
                continue
            slot = d * self.cap + int(self.running[d])
            self.send_pk[slot * self.stride:(slot + 1) * self.stride] = a[k]
            self.send_ln[slot] = ln[k]
            self.running[d] += 1


def _worker(rank, world, port, result_q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import oracle_ffi as O
    import sar_inputs as S
    import e2sar_amd.dist as D

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        D.RegionRouter = _FakeRouter
        mp_ = O.max_pld_len(1500)
        stride = (36 + mp_ + 15) // 16 * 16
        evs = [S.event_bytes(i, 5000 + 3119 * i) for i in range(8)]
        pks, lns = [], []
        for i, e in enumerate(evs):
            p, l = O.segment_event(e, i, S.DATA_ID, S.entropy(i), S.lb_tick(i), 2, mp_, stride)
            pks.append(p)
            lns.append(l)
        allp = np.concatenate(pks)
        alll = np.concatenate(lns)
        landed = np.arange(len(alll)) % world == rank
        lp, ll = allp[landed], alll[landed].astype(np.int32)
        n = len(ll)
        cuts = [0, n // 3, (2 * n) // 3 + 1, n]
        R = _FakeR(world, rank, stride)
        pipe = D.SpreadPipeline(_Ctx(), R, stride, max(b - a for a, b in zip(cuts[:-1], cuts[1:])), world, rank)
        pipe.begin_step()
        for a, b in zip(cuts[:-1], cuts[1:]):
            pipe.land(torch.from_numpy(lp[a:b].reshape(-1).copy()), torch.from_numpy(ll[a:b].copy()), b - a)
        pipe.flush()
        mine = sorted(bytes(allp[k, : alll[k]]) for k in range(len(alll)) if _ev_of(allp[k]) % world == rank)
        got = sorted(R.in_place + R.received)
        result_q.put((rank, got == mine, len(R.in_place), len(R.received), pipe.sent, pipe.received,
                      pipe.matrices, [c for _, c in pipe.recv_log]))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_spread_pipeline_gloo(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=120) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    for rank, ok, n_in, n_rx, sent, received, mats, rlog in res:
        assert ok, (rank, n_in, n_rx)
        assert n_rx == received == sum(rlog) and len(mats) == 3
    # every batch's count matrix is the same on every rank, and what rank s sends rank d is
    # what d receives from s
    assert all(r[6] == res[0][6] for r in res)
    assert sum(r[4] for r in res) == sum(r[5] for r in res) > 0
