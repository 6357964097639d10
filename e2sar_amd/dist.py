"""Multi-GPU SAR: events are owned by rank ``eventNum % world``.

Normal operation needs no communication: each GPU segments and reassembles the events it
owns.  When datagrams *land* on a rank that does not own their event (a modelled NIC /
RSS spread), each rank

1. reassembles the datagrams it owns where they landed (``DeviceReassembler.set_owner``:
   the reassembler skips other ranks' events, so nothing of its own is copied twice);
2. packs the foreign ones into per-owner spans on the GPU (``PacketRouter.route`` with
   ``foreign_only=True``: gfx950 route kernels behind e2sar_hip_route_foreign);
3. ``exchange`` moves the spans with one all-to-all-v (the split sizes come from one
   all-gather of the per-rank count vectors: one host read per exchange);
4. reassembles what it received.

With the ``nccl`` backend (RCCL on ROCm) the transfer runs over xGMI, peer to peer, not as
a ring.  The reference never needs this step -- its load balancer steers every fragment of
an event to one receiver (e2sarDPSegmenter.hpp:231-235), and the receiver keys its
threads by the same eventNum (e2sarDPReassembler.hpp:224-229) -- so there is no reference
call pattern to mirror.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist


def owner(event_num: int, world: int) -> int:
    return int(event_num) % int(world)


def _via_host(group, t: torch.Tensor) -> bool:
    """gloo's collectives take host tensors (device tensors are staged through host memory)
    and have no list all-to-all: with gloo every exchange goes through all_to_all_single on
    host tensors."""
    return dist.get_backend(group) == "gloo"


def count_matrix(counts: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> List[List[int]]:
    """m[s][d] = datagrams rank s sends rank d, from every rank's count vector (on the
    device): one all-gather of the world x world matrix, then ONE host read."""
    world = dist.get_world_size(group)
    if counts.numel() != world:
        raise ValueError("counts must have one entry per rank")
    c = counts.to(torch.int64)
    if _via_host(group, c):
        c = c.cpu()
    rows = [torch.empty_like(c) for _ in range(world)]
    dist.all_gather(rows, c, group=group)
    return [[int(x) for x in row] for row in torch.stack(rows).tolist()]    # the one host read


def exchange_counts(counts: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> Tuple[List[int], List[int]]:
    """(send, recv) split sizes of this rank (count_matrix's row and column)."""
    m = count_matrix(counts, group)
    rank = dist.get_rank(group)
    return m[rank], [m[s][rank] for s in range(len(m))]


def exchange(send_pk: torch.Tensor, send_ln: torch.Tensor, counts: Union[Sequence[int], torch.Tensor], stride: int,
             group: Optional[dist.ProcessGroup] = None,
             out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> Tuple[torch.Tensor, torch.Tensor, int]:
    """All-to-all-v of datagram slots.

    send_pk: uint8, sum(counts)*stride bytes, the span for rank d at offset
    sum(counts[:d])*stride; send_ln: int32 lengths in the same order; counts: datagrams per
    destination rank, either the route kernels' device vector (split sizes by
    ``exchange_counts``: one host read) or host ints (receive sizes by an all-to-all of
    the counts).  out: optional preallocated (recv_pk, recv_ln) used when large enough, so
    a steady stream of batches does not allocate per call.  Returns (recv_pk, recv_ln,
    n_recv), spans ordered by source rank.  Backends: nccl (RCCL) on device tensors; gloo,
    whose all-to-all takes host tensors, through host staging copies (the CPU rehearsal path).
    """
    world = dist.get_world_size(group)
    dev = send_pk.device
    via_host = _via_host(group, send_pk)
    anything = True
    if isinstance(counts, torch.Tensor):
        m = count_matrix(counts, group)
        rank = dist.get_rank(group)
        sc, rc = m[rank], [m[s][rank] for s in range(world)]
        anything = any(any(row) for row in m)
    else:
        sc = [int(x) for x in counts]
        if len(sc) != world:
            raise ValueError("counts must have one entry per rank")
        cdev = torch.device("cpu") if via_host else dev
        cnt = torch.tensor(sc, dtype=torch.int64, device=cdev)
        rcnt = torch.empty_like(cnt)
        dist.all_to_all_single(rcnt, cnt, group=group)
        rc = [int(x) for x in rcnt.tolist()]
    n_recv = sum(rc)
    if out is not None and out[0].numel() >= n_recv * stride and out[1].numel() >= n_recv and out[0].device == dev:
        recv_pk, recv_ln = out
    else:
        recv_pk = torch.empty(max(n_recv, 1) * stride, dtype=torch.uint8, device=dev)
        recv_ln = torch.empty(max(n_recv, 1), dtype=torch.int32, device=dev)
    n_send = sum(sc)
    if not anything:
        return recv_pk, recv_ln, 0                          # no rank sends anything: skip the collective
    spk, sln = send_pk[: n_send * stride], send_ln[:n_send]
    rpk, rln = recv_pk[: n_recv * stride], recv_ln[:n_recv]
    if via_host:
        hpk, hln = torch.empty(n_recv * stride, dtype=torch.uint8), torch.empty(n_recv, dtype=torch.int32)
        dist.all_to_all_single(hpk, spk.cpu(), [c * stride for c in rc], [c * stride for c in sc], group=group)
        dist.all_to_all_single(hln, sln.cpu(), rc, sc, group=group)
        rpk.copy_(hpk)
        rln.copy_(hln)
    else:
        dist.all_to_all_single(rpk, spk, [c * stride for c in rc], [c * stride for c in sc], group=group)
        dist.all_to_all_single(rln, sln, rc, sc, group=group)
    return recv_pk, recv_ln, n_recv


def exchange_regions(send_pk: torch.Tensor, send_ln: torch.Tensor, running: torch.Tensor, cap: int, stride: int,
                     group: Optional[dist.ProcessGroup] = None,
                     out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                     m: Optional[List[List[int]]] = None) -> Tuple[torch.Tensor, torch.Tensor, int]:
    """All-to-all-v of per-rank regions filled by ``RegionRouter``: rank d's datagrams are
    the first running[d] slots of region d (slots [d*cap, d*cap + running[d]) of send_pk /
    send_ln).  Split sizes from one all-gather of the running counters (one host read).
    nccl: one all_to_all over the region views (RCCL send/recv per peer, no packing copy);
    gloo: the regions are gathered on the host and sent with all_to_all_single.  Returns
    (recv_pk, recv_ln, n_recv), received spans contiguous in source-rank order.  m: the
    count matrix when the caller already gathered it."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if m is None:
        m = count_matrix(running, group)
    if any(c > cap for row in m for c in row):
        raise RuntimeError(f"route regions overflowed (cap {cap} datagrams per rank): {m}")
    sc, rc = m[rank], [m[s][rank] for s in range(world)]
    n_recv = sum(rc)
    dev = send_pk.device
    if out is not None and out[0].numel() >= n_recv * stride and out[1].numel() >= n_recv and out[0].device == dev:
        recv_pk, recv_ln = out
    else:
        recv_pk = torch.empty(max(n_recv, 1) * stride, dtype=torch.uint8, device=dev)
        recv_ln = torch.empty(max(n_recv, 1), dtype=torch.int32, device=dev)
    if not any(any(row) for row in m):
        return recv_pk, recv_ln, 0                          # no rank sends anything: skip the collective
    roff = [sum(rc[:s]) for s in range(world)]
    if _via_host(group, send_pk):
        spk = torch.cat([send_pk[d * cap * stride:(d * cap + sc[d]) * stride].cpu() for d in range(world)])
        sln = torch.cat([send_ln[d * cap:d * cap + sc[d]].cpu() for d in range(world)])
        hpk, hln = torch.empty(n_recv * stride, dtype=torch.uint8), torch.empty(n_recv, dtype=torch.int32)
        dist.all_to_all_single(hpk, spk, [c * stride for c in rc], [c * stride for c in sc], group=group)
        dist.all_to_all_single(hln, sln, rc, sc, group=group)
        recv_pk[: n_recv * stride].copy_(hpk)
        recv_ln[:n_recv].copy_(hln)
    else:
        dist.all_to_all([recv_pk[roff[s] * stride:(roff[s] + rc[s]) * stride] for s in range(world)],
                        [send_pk[d * cap * stride:(d * cap + sc[d]) * stride] for d in range(world)], group=group)
        dist.all_to_all([recv_ln[roff[s]:roff[s] + rc[s]] for s in range(world)],
                        [send_ln[d * cap:d * cap + sc[d]] for d in range(world)], group=group)
    return recv_pk, recv_ln, n_recv


class RegionRouter:
    """Routes a stream of landed batches, one launch per batch, into per-rank regions of
    cap datagram slots (e2sar_hip_route_append); ``exchange_regions`` sends them once per
    step.  Routing a batch right after it landed reads it from the Infinity Cache."""

    def __init__(self, ctx, stride: int, cap: int, max_batch: int, world: int, rank: int,
                 with_lb_header: bool = True, foreign_only: bool = True):
        from ._capi import lib
        self.ctx = ctx
        self.stride, self.cap, self.world, self.rank = stride, cap, world, rank
        self.with_lb, self.foreign_only, self.max_batch = with_lb_header, foreign_only, max_batch
        d = ctx.torch_device
        self.send_pk = torch.empty(world * cap * stride, dtype=torch.uint8, device=d)
        self.send_ln = torch.empty(world * cap, dtype=torch.int32, device=d)
        self.running = torch.zeros(world, dtype=torch.int32, device=d)
        ws = int(lib().e2sar_hip_route_workspace_bytes(max_batch, world))
        self.workspace = torch.empty(max(ws, 16), dtype=torch.uint8, device=d)

    def reset(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Empty the regions (a fill kernel on the stream, default the current one: capture-safe)."""
        from ._capi import check, lib
        from .sar import _stream_handle
        check(lib().e2sar_hip_memset_async(self.ctx.handle, C.c_void_p(self.running.data_ptr()), 0,
                                           self.running.numel() * 4, C.c_void_p(_stream_handle(stream))))

    def route(self, pk: torch.Tensor, ln: torch.Tensor, n: int, stream: Optional[torch.cuda.Stream] = None):
        from ._capi import check, lib
        from .sar import _stream_handle
        if n > self.max_batch:
            raise ValueError("batch larger than the router was sized for")
        check(lib().e2sar_hip_route_append(
            self.ctx.handle, C.c_void_p(pk.data_ptr()), self.stride, C.c_void_p(ln.data_ptr()), n,
            1 if self.with_lb else 0, self.world, self.rank, 1 if self.foreign_only else 0,
            C.c_void_p(self.send_pk.data_ptr()), C.c_void_p(self.send_ln.data_ptr()), self.cap,
            C.c_void_p(self.running.data_ptr()), C.c_void_p(self.workspace.data_ptr()), self.workspace.numel(),
            C.c_void_p(_stream_handle(stream))))

    def exchange(self, group: Optional[dist.ProcessGroup] = None,
                 out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
        return exchange_regions(self.send_pk, self.send_ln, self.running, self.cap, self.stride, group, out)


class PacketRouter:
    """Packs a landed datagram batch into per-owner spans on the GPU."""

    def __init__(self, ctx, stride: int, max_packets: int, world: int, rank: int, with_lb_header: bool = True):
        from ._capi import lib
        self.ctx = ctx
        self.stride = stride
        self.world = world
        self.rank = rank
        self.with_lb = with_lb_header
        self.max_packets = max_packets
        d = ctx.torch_device
        self.send_pk = torch.empty(max(max_packets, 1) * stride, dtype=torch.uint8, device=d)
        self.send_ln = torch.empty(max(max_packets, 1), dtype=torch.int32, device=d)
        self.counts = torch.zeros(world, dtype=torch.int32, device=d)
        ws = int(lib().e2sar_hip_route_workspace_bytes(max_packets, world))
        self.workspace = torch.empty(max(ws, 16), dtype=torch.uint8, device=d)

    def route(self, pk: torch.Tensor, ln: torch.Tensor, n: int, stream: Optional[torch.cuda.Stream] = None,
              foreign_only: bool = False):
        """Returns (send_pk, send_ln, counts) with counts still on the device.  foreign_only:
        pack only datagrams other ranks own (e2sar_hip_route_foreign); the rest stay for a
        reassembler set to this rank's ownership."""
        from ._capi import check, lib
        from .sar import _stream_handle
        if n > self.max_packets:
            raise ValueError("batch larger than the router was sized for")
        fn = lib().e2sar_hip_route_foreign if foreign_only else lib().e2sar_hip_route_batch
        check(fn(
            self.ctx.handle, C.c_void_p(pk.data_ptr()), self.stride, C.c_void_p(ln.data_ptr()), n,
            1 if self.with_lb else 0, self.world, self.rank, C.c_void_p(self.send_pk.data_ptr()),
            C.c_void_p(self.send_ln.data_ptr()), C.c_void_p(self.counts.data_ptr()),
            C.c_void_p(self.workspace.data_ptr()), self.workspace.numel(), C.c_void_p(_stream_handle(stream))))
        return self.send_pk, self.send_ln, self.counts


class SpreadPipeline:
    """BASELINE config 4 per landed batch, with the exchange overlapped.

    For each batch that lands on this rank (``land``), on the caller's stream:

    1. the datagrams this rank owns are reassembled where they landed (``R`` must be set to
       this rank's ownership, ``DeviceReassembler.set_owner``), while the batch is still in
       the Infinity Cache;
    2. the foreign ones are appended to per-owner regions (``RegionRouter``, one launch);

    then, on the communication stream, the per-owner counts are all-gathered (RCCL) and
    copied to pinned host memory.  The host reads batch b's counts only after it has queued
    batch b + depth - 1's landing work, then issues batch b's ``all_to_all`` of the regions
    (RCCL, peer to peer over xGMI) on the same stream and the reassembly of what arrived
    (classify + scatter with streaming loads) on a second stream.  So batch b's exchange and
    the reassembly of what it brought run while later batches land and are reassembled in
    place, and the step costs max(landing, exchange) instead of their sum.  ``depth``
    region / receive buffer sets rotate; a set is reused only after the exchange and
    reassembly that read it have finished (stream events, no host wait).

    Every collective -- count all-gathers and exchanges alike -- goes through ONE
    communicator on ONE stream, in one order that every rank issues identically (each
    land(): the exchange of batch b - depth + 1, then the count gather of batch b).  RCCL,
    like NCCL, does not promise progress for collectives of two communicators in flight at
    once, so nothing here depends on it: the stream serialises the collectives in the order
    every rank enqueued them.  The cost is that batch b's count gather queues behind batch
    b - depth + 1's exchange, so the host, reading b's counts depth - 1 landings later,
    waits only when the exchange has fallen depth - 1 batches behind the landing.

    With gloo (the CPU / one-GPU rehearsal) every exchange is synchronous through host
    memory and the received datagrams are reassembled on the caller's stream.

    The reference needs no exchange: its load balancer steers every fragment of an event to
    one receiver (e2sarDPSegmenter.hpp:231-233, e2sarDPReassembler.hpp:223-229).
    """

    def __init__(self, ctx, R, stride: int, max_batch: int, world: int, rank: int,
                 group: Optional[dist.ProcessGroup] = None, depth: int = 3, with_lb_header: bool = True,
                 in_place: bool = True):
        """in_place=False routes every landed datagram, this rank's own included, through the
        exchange (no in-place reassembly): the route-all form, which also drives the whole
        RCCL data path at world 1."""
        if depth < 2:
            # a region set is reused only after the exchange that reads it was issued, which
            # happens one land() later: with one set, land() would reset and refill it under
            # the previous batch's pending all_to_all
            raise ValueError("SpreadPipeline needs depth >= 2 (region / receive sets in rotation)")
        self.ctx, self.R, self.stride, self.max_batch = ctx, R, stride, max_batch
        self.world, self.rank, self.group, self.depth = world, rank, group, depth
        self.in_place = in_place
        dev = ctx.torch_device
        self.active = world > 1 or not in_place
        self.nccl = self.active and dist.get_backend(group) == "nccl"
        self.routers = [RegionRouter(ctx, stride, max_batch, max_batch, world, rank, with_lb_header,
                                     foreign_only=in_place) for _ in range(depth)] if self.active else []
        # a batch can bring at most every peer's whole batch (and its own, routing all)
        rcap = max(1, (world - (1 if in_place else 0)) * max_batch)
        self.recv = [(torch.empty(rcap * stride, dtype=torch.uint8, device=dev),
                      torch.empty(rcap, dtype=torch.int32, device=dev)) for _ in range(depth)] if self.active else []
        self.work = [R.alloc_work(rcap) for _ in range(depth)] if self.active else []
        self.comm = torch.cuda.Stream(dev) if self.nccl else None
        self.rx = torch.cuda.Stream(dev) if self.nccl else None
        self.lag = depth - 1                  # batches whose exchange is still to be issued
        self.mat_dev = [torch.zeros(world * world, dtype=torch.int32, device=dev) for _ in range(depth)]
        self.mat_host = [torch.zeros(world * world, dtype=torch.int32).pin_memory() for _ in range(depth)] \
            if self.nccl else []
        mk = (lambda: torch.cuda.Event()) if self.nccl else (lambda: None)
        self.ev_routed = [mk() for _ in range(depth)]
        self.ev_cnt = [mk() for _ in range(depth)]
        self.ev_a2a = [mk() for _ in range(depth)]       # region set free again
        self.ev_rx = [mk() for _ in range(depth)]        # receive set free again
        self.used = [False] * depth
        self.now_ms = 0
        self.pending: List[int] = []
        self.nb = 0
        self.sent = 0            # foreign datagrams sent / received since begin_step
        self.received = 0
        self.matrices: List[List[List[int]]] = []
        self.recv_log: List[Tuple[int, int]] = []        # (receive set, datagrams) per batch
        # timing hook: timed(name, stream, fn, *a, **kw) -> fn(*a, stream=stream, **kw)
        self.timed = lambda name, stream, fn, *a, **kw: fn(*a, stream=stream, **kw)

    def begin_step(self) -> None:
        self.sent = self.received = 0
        self.matrices = []
        self.recv_log = []

    def land(self, pk: torch.Tensor, ln: torch.Tensor, n: int, now_ms: int = 0) -> None:
        """One landed batch (on the current stream): in-place reassembly of the owned
        datagrams, routing of the foreign ones, and the exchange pipeline's next stage."""
        main = torch.cuda.current_stream() if torch.cuda.is_available() else None
        self.now_ms = now_ms
        if self.in_place:
            self.timed("reas_kernel", main, self.R.reassemble, pk, self.stride, ln, n, now_ms=now_ms)
        if not self.active:
            return
        slot = self.nb % self.depth
        self.nb += 1
        router = self.routers[slot]
        if self.nccl and self.used[slot]:
            main.wait_event(self.ev_a2a[slot])          # the region set's last exchange has read it
        router.reset(stream=main)
        self.timed("route_kernels", main, router.route, pk, ln, n)
        self.used[slot] = True
        if not self.nccl:
            self._exchange_sync(slot, main)
            return
        self.ev_routed[slot].record(main)
        # exchange the batch landed depth - 1 batches ago, then gather this batch's counts:
        # both on the one communication stream and communicator, in this order on every rank
        while len(self.pending) >= self.lag:
            self._finish(self.pending.pop(0))
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(self.ev_routed[slot])
            dist.all_gather_into_tensor(self.mat_dev[slot], router.running, group=self.group)
            self.mat_host[slot].copy_(self.mat_dev[slot], non_blocking=True)
            self.ev_cnt[slot].record(self.comm)
        self.pending.append(slot)

    def _counts(self, m: List[List[int]]):
        if any(c > self.max_batch for row in m for c in row):
            raise RuntimeError(f"route regions overflowed (cap {self.max_batch} datagrams per rank): {m}")
        sc, rc = m[self.rank], [m[s][self.rank] for s in range(self.world)]
        self.sent += sum(c for d, c in enumerate(sc) if d != self.rank)
        self.received += sum(c for s, c in enumerate(rc) if s != self.rank)
        self.matrices.append(m)
        return sc, rc

    def _finish(self, slot: int) -> None:
        """Batch of region set `slot`: read its counts (host), exchange, reassemble arrivals.
        Called depth - 1 batches after the batch landed; its count gather was queued behind
        the exchange issued depth - 1 batches before it, so the wait below blocks only while
        the exchanges run more than depth - 1 batches behind the landing."""
        self.ev_cnt[slot].synchronize()
        flat = self.mat_host[slot].tolist()
        W = self.world
        m = [flat[s * W:(s + 1) * W] for s in range(W)]
        sc, rc = self._counts(m)
        router = self.routers[slot]
        rpk, rln = self.recv[slot]
        n_recv = sum(rc)
        st = self.stride
        cap = self.max_batch
        roff = [sum(rc[:s]) for s in range(W)]
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(self.ev_rx[slot])       # the receive set's last reassembly has read it
            if any(any(row) for row in m):
                def a2a(stream=None):
                    dist.all_to_all([rpk[roff[s] * st:(roff[s] + rc[s]) * st] for s in range(W)],
                                    [router.send_pk[d * cap * st:(d * cap + sc[d]) * st] for d in range(W)],
                                    group=self.group)
                    dist.all_to_all([rln[roff[s]:roff[s] + rc[s]] for s in range(W)],
                                    [router.send_ln[d * cap:d * cap + sc[d]] for d in range(W)], group=self.group)
                self.timed("exchange", self.comm, a2a)
            self.ev_a2a[slot].record(self.comm)
        self.recv_log.append((slot, n_recv))
        if n_recv:
            self.rx.wait_event(self.ev_a2a[slot])
            self._reassemble_received(rpk, rln, n_recv, self.work[slot], self.rx)
        self.ev_rx[slot].record(self.rx)

    def _reassemble_received(self, rpk, rln, n, work, stream) -> None:
        self.timed("reas_classify_kernel", stream, self.R.classify, rpk, self.stride, rln, n, work,
                   now_ms=self.now_ms)
        self.timed("reas_scatter_kernel", stream, self.R.scatter, rpk, self.stride, n, work)

    def _exchange_sync(self, slot: int, main) -> None:
        router = self.routers[slot]
        m = count_matrix(router.running, self.group)
        self._counts(m)
        res = []

        def ex(stream=None):
            res.append(exchange_regions(router.send_pk, router.send_ln, router.running, self.max_batch,
                                        self.stride, self.group, out=self.recv[slot], m=m))
        self.timed("exchange", main, ex)
        rpk, rln, n = res[0]
        self.recv_log.append((slot, n))
        if n:
            self._reassemble_received(rpk, rln, n, self.work[slot], main)

    def flush(self) -> None:
        """Finish every batch's exchange and reassembly; the current stream waits for them."""
        while self.pending:
            self._finish(self.pending.pop(0))
        if self.nccl:
            main = torch.cuda.current_stream()
            main.wait_stream(self.comm)
            main.wait_stream(self.rx)
