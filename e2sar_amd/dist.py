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
    """gloo's collectives take host tensors: device tensors are staged through host memory."""
    return dist.get_backend(group) == "gloo" and t.is_cuda


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
                     out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> Tuple[torch.Tensor, torch.Tensor, int]:
    """All-to-all-v of per-rank regions filled by ``RegionRouter``: rank d's datagrams are
    the first running[d] slots of region d (slots [d*cap, d*cap + running[d]) of send_pk /
    send_ln).  Split sizes from one all-gather of the running counters (one host read).
    nccl: one all_to_all over the region views (RCCL send/recv per peer, no packing copy);
    gloo: the regions are gathered on the host and sent with all_to_all_single.  Returns
    (recv_pk, recv_ln, n_recv), received spans contiguous in source-rank order."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
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
