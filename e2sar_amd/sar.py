"""Device-level SAR API over the C ABI (``include/e2sar_hip.h``).

``DeviceSegmenter`` and ``DeviceReassembler`` are thin, allocation-aware wrappers: event
bytes, datagrams and reassembled events stay in HBM; torch is used only as the device
memory / stream plumbing.  The reference-shaped ``Segmenter``/``Reassembler`` classes
(``e2sar_amd.dataplane``) are built on top of these.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _capi
from ._capi import check, lib


def _stream_handle(stream: Optional[torch.cuda.Stream]) -> int:
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


def total_hdr_len(use_ipv6: bool = False) -> int:
    """IP + UDP + LB + RE header bytes (e2sarHeaders.hpp:419-421): 64 / 84."""
    return int(lib().e2sar_hip_total_hdr_len(1 if use_ipv6 else 0))


def max_pld_len(mtu: int, use_ipv6: bool = False) -> int:
    """Segmenter maxPldLen = mtu - total header (e2sarDPSegmenter.hpp:241)."""
    return int(lib().e2sar_hip_max_pld_len(mtu, 1 if use_ipv6 else 0))


def num_packets(nbytes: int, max_pld: int) -> int:
    """ceil(bytes / maxPldLen) (e2sarDPSegmenter.cpp:670)."""
    return int(lib().e2sar_hip_num_packets(nbytes, max_pld))


def packet_stride(max_pld: int) -> int:
    return int(lib().e2sar_hip_packet_stride(max_pld))


class Context:
    """A device + stream binding (e2sar_hip_ctx)."""

    def __init__(self, device: int = 0, stream: Optional[torch.cuda.Stream] = None):
        torch.cuda.set_device(device)
        self.device = device
        self.torch_device = torch.device("cuda", device)
        self.stream = stream if stream is not None else torch.cuda.current_stream(device)
        h = C.c_void_p()
        check(lib().e2sar_hip_ctx_create(device, C.c_void_p(int(self.stream.cuda_stream)), C.byref(h)))
        self._h = h

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def sync(self) -> None:
        check(lib().e2sar_hip_ctx_sync(self._h))

    def copy_spans(self, spans: Sequence[tuple], stream: Optional[torch.cuda.Stream] = None) -> None:
        """(src_ptr, dst_ptr, nbytes) spans, device or pinned host memory, copied by
        e2sar_hip_copy_spans (one launch per 64 spans)."""
        arr = (_capi.CopySpan * max(1, len(spans)))()
        for k, (a, b, n) in enumerate(spans):
            arr[k] = _capi.CopySpan(int(a), int(b), int(n))
        check(lib().e2sar_hip_copy_spans(self._h, arr, len(spans), C.c_void_p(_stream_handle(stream))))

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().e2sar_hip_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class SegPlan:
    """Host event table + its device copy for one segment batch."""
    host: "C.Array"
    device: torch.Tensor          # uint8 tensor holding the e2sar_hip_seg_event table
    n_events: int
    total_packets: int
    max_packets_per_event: int
    aligned4: bool


class DeviceSegmenter:
    """Segments batches of device-resident events into device-resident datagrams.

    Replaces SendThreadState::_send's fragment loop (e2sarDPSegmenter.cpp:660-871):
    every datagram is [LB header][RE header][payload slice] exactly as the reference
    emits it; the socket send is the caller's business (or the datagrams stay in HBM).
    """

    def __init__(self, ctx: Context, mtu: int = 1500, use_ipv6: bool = False, lb_hdr_version: int = 2):
        self.ctx = ctx
        self.mtu = mtu
        self.max_pld = max_pld_len(mtu, use_ipv6)
        if mtu > 9000:
            raise ValueError("MTU set too long, limit 9000")       # hpp:310-311
        if self.max_pld == 0:
            raise ValueError("Insufficient MTU length to accommodate headers")  # hpp:315-316
        self.stride = packet_stride(self.max_pld)
        self.lb_hdr_version = lb_hdr_version

    def plan(self, events: Sequence[tuple]) -> SegPlan:
        """events: (data_ptr, nbytes, eventNum, dataId, entropy, lbTick) tuples, data on device."""
        n = len(events)
        arr = (_capi.SegEvent * max(n, 1))()
        aligned4 = True
        for k, (ptr, nbytes, evn, did, ent, tick) in enumerate(events):
            if nbytes >= 1 << 32:
                raise ValueError("event larger than 4 GiB (REHdr bufferLength is u32)")
            e = arr[k]
            e.data = int(ptr)
            e.bytes = int(nbytes)
            e.eventNum = int(evn) & (2**64 - 1)
            e.dataId = int(did) & 0xFFFF
            e.entropy = int(ent) & 0xFFFF
            e.lbTick = int(tick) & (2**64 - 1)
            aligned4 = aligned4 and (int(ptr) % 4 == 0)
        tot = C.c_uint32()
        mx = C.c_uint32()
        check(lib().e2sar_hip_seg_plan(arr, n, self.max_pld, C.byref(tot), C.byref(mx)))
        raw = np.frombuffer(bytes(arr)[: n * C.sizeof(_capi.SegEvent)], dtype=np.uint8).copy()
        dev = torch.from_numpy(raw).to(self.ctx.torch_device, non_blocking=False)
        return SegPlan(arr, dev, n, int(tot.value), int(mx.value), aligned4)

    def groups(self, plan: SegPlan):
        """The reassembly groups that match this segmenter's XCD stripes for `plan`
        (e2sar_hip_seg_groups): (device uint32 tensor of starts, nGroups), or (None, 0)
        when the batch has no stripes.  For DeviceReassembler.reassemble_groups."""
        spc = self.stride // 16
        units = plan.n_events * max(1, (plan.max_packets_per_event * spc + 511) // 512)
        cap = units + 2
        starts = (C.c_uint32 * cap)()
        ng = C.c_uint32()
        _capi.need_experimental("DeviceSegmenter.groups")
        check(lib().e2sar_hip_seg_groups(plan.host, plan.n_events, plan.max_packets_per_event, self.max_pld,
                                         self.stride, starts, cap, C.byref(ng)))
        if ng.value == 0:
            return None, 0
        host = np.frombuffer(bytes(starts), dtype=np.uint32)[: ng.value + 1].copy()
        return torch.from_numpy(host.view(np.int32)).to(self.ctx.torch_device), int(ng.value)

    def alloc_packets(self, n_packets: int):
        pk = torch.empty(max(n_packets, 1) * self.stride, dtype=torch.uint8, device=self.ctx.torch_device)
        ln = torch.empty(max(n_packets, 1), dtype=torch.int32, device=self.ctx.torch_device)
        return pk, ln

    def segment(self, plan: SegPlan, packets: torch.Tensor, lens: Optional[torch.Tensor],
                stream: Optional[torch.cuda.Stream] = None, recycle: Optional["DeviceReassembler"] = None,
                force: bool = False) -> int:
        """recycle: also recycle that reassembler (as DeviceReassembler.recycle(force)) in the
        same launch (e2sar_hip_segment_batch_recycle)."""
        if packets.numel() < plan.total_packets * self.stride:
            raise ValueError("packet buffer too small")
        common = (C.c_void_p(plan.device.data_ptr()), plan.n_events,
                  plan.max_packets_per_event, self.lb_hdr_version, self.max_pld,
                  1 if plan.aligned4 else 0, C.c_void_p(packets.data_ptr()), self.stride,
                  C.c_void_p(lens.data_ptr() if lens is not None else 0))
        if recycle is not None:
            check(lib().e2sar_hip_segment_batch_recycle(self.ctx.handle, *common, recycle.handle, 1 if force else 0,
                                                        C.c_void_p(_stream_handle(stream))))
        else:
            check(lib().e2sar_hip_segment_batch(self.ctx.handle, *common, C.c_void_p(_stream_handle(stream))))
        return plan.total_packets

    def segment_reassemble(self, plan: SegPlan, packets: torch.Tensor, lens: torch.Tensor,
                           reas: "DeviceReassembler", now_ms: int = 0,
                           stream: Optional[torch.cuda.Stream] = None) -> int:
        """Chained form: segment the batch and reassemble the same datagrams into `reas`
        in one launch (e2sar_hip_segment_reassemble_batch)."""
        if packets.numel() < plan.total_packets * self.stride or lens.numel() < plan.total_packets:
            raise ValueError("packet buffer too small")
        _capi.need_experimental("DeviceSegmenter.segment_reassemble")
        check(lib().e2sar_hip_segment_reassemble_batch(
            self.ctx.handle, C.c_void_p(plan.device.data_ptr()), plan.n_events, plan.max_packets_per_event,
            plan.total_packets, self.lb_hdr_version, self.max_pld, C.c_void_p(packets.data_ptr()), self.stride,
            C.c_void_p(lens.data_ptr()), reas._h, int(now_ms), C.c_void_p(_stream_handle(stream))))
        return plan.total_packets

    def segment_reassemble_batches(self, plans: Sequence[SegPlan], bufs: Sequence[tuple],
                                   reas: "DeviceReassembler", now_ms: int = 0,
                                   stream: Optional[torch.cuda.Stream] = None) -> int:
        """Chained form over several batches in one launch (at most 8;
        e2sar_hip_segment_reassemble_batches); bufs[k] = (packets, lens) of plans[k], all distinct."""
        arr = (_capi.SegReasBatch * max(1, len(plans)))()
        for k, (p, (pk, ln)) in enumerate(zip(plans, bufs)):
            if pk.numel() < p.total_packets * self.stride or ln.numel() < p.total_packets:
                raise ValueError("packet buffer too small")
            arr[k] = _capi.SegReasBatch(p.device.data_ptr(), pk.data_ptr(), ln.data_ptr(), p.n_events,
                                        p.max_packets_per_event, p.total_packets, 0)
        _capi.need_experimental("DeviceSegmenter.segment_reassemble_batches")
        check(lib().e2sar_hip_segment_reassemble_batches(
            self.ctx.handle, arr, len(plans), self.lb_hdr_version, self.max_pld, self.stride, reas._h, int(now_ms),
            C.c_void_p(_stream_handle(stream))))
        return sum(p.total_packets for p in plans)

    def segment_device(self, events: torch.Tensor, counts: torch.Tensor, max_events: int,
                       max_packets_per_event: int, packets: torch.Tensor, lens: Optional[torch.Tensor],
                       stream: Optional[torch.cuda.Stream] = None) -> None:
        """Segment a descriptor table built on the device (DeviceReassembler.relay_plan):
        the event count is counts[0], read by the kernel; max_events bounds it."""
        if packets.numel() < max_events * max_packets_per_event * self.stride:
            raise ValueError("packet buffer too small for the bound")
        check(lib().e2sar_hip_segment_batch_dev(
            self.ctx.handle, C.c_void_p(events.data_ptr()), C.c_void_p(counts.data_ptr()), max_events,
            max_packets_per_event, self.lb_hdr_version, self.max_pld, C.c_void_p(packets.data_ptr()),
            self.stride, C.c_void_p(lens.data_ptr() if lens is not None else 0),
            C.c_void_p(_stream_handle(stream))))


SEG_EVENT_BYTES = 40       # sizeof(e2sar_hip_seg_event)


class DeviceReassembler:
    """Reassembles device-resident datagram batches into a device event arena.

    Replaces the per-packet body of RecvThreadState::_threadBody
    (e2sarDPReassembler.cpp:310-428), the eventsInProgress map and the event queue.
    """

    def __init__(self, ctx: Context, with_lb_header: bool = False, table_slots: int = 4096,
                 queue_capacity: int = 4096, lost_capacity: int = 4096, arena_bytes: int = 1 << 30,
                 compactable: bool = False, flags: int = 0, group_size: int = 0):
        """group_size: datagrams per fused-kernel workgroup (1..64), 0 = automatic."""
        self.ctx = ctx
        flags |= _capi.REAS_COMPACTABLE if compactable else 0
        cfg = _capi.ReasConfig(1 if with_lb_header else 0, table_slots, queue_capacity,
                               lost_capacity, arena_bytes, flags, group_size)
        h = C.c_void_p()
        check(lib().e2sar_hip_reas_create(ctx.handle, C.byref(cfg), C.byref(h)))
        self._h = h
        self.with_lb_header = with_lb_header
        self.arena_bytes = arena_bytes
        self.arena_ptr = int(lib().e2sar_hip_reas_arena(h) or 0)
        self._evbuf = (_capi.EventRec * queue_capacity)()
        self._lostbuf = (_capi.LostRec * lost_capacity)()

    @property
    def handle(self):
        return self._h

    def set_owner(self, world: int, rank: int) -> None:
        """Take only events with eventNum % world == rank (e2sar_hip_reas_set_owner)."""
        check(lib().e2sar_hip_reas_set_owner(self._h, int(world), int(rank)))

    def set_cold(self, cold: bool) -> None:
        """Streaming datagram loads for the following launches (e2sar_hip_reas_set_cold)."""
        check(lib().e2sar_hip_reas_set_cold(self._h, 1 if cold else 0))

    def reassemble(self, packets: torch.Tensor, stride: int, lens: torch.Tensor, n: int,
                   now_ms: int = 0, stream: Optional[torch.cuda.Stream] = None) -> None:
        if n == 0:
            return
        if lens.numel() < n or packets.numel() < n * stride:
            raise ValueError("packet batch buffers too small")
        check(lib().e2sar_hip_reassemble_batch(
            self._h, C.c_void_p(packets.data_ptr()), stride, C.c_void_p(lens.data_ptr()), n,
            int(now_ms), C.c_void_p(_stream_handle(stream))))

    def reassemble_groups(self, packets: torch.Tensor, stride: int, lens: torch.Tensor, n: int,
                          starts: Optional[torch.Tensor], n_groups: int, now_ms: int = 0,
                          stream: Optional[torch.cuda.Stream] = None) -> None:
        """reassemble() over a group table (DeviceSegmenter.groups: the XCD stripes the batch
        was segmented in), e2sar_hip_reassemble_groups."""
        if n == 0:
            return
        if lens.numel() < n or packets.numel() < n * stride:
            raise ValueError("packet batch buffers too small")
        if starts is not None and starts.numel() < n_groups + 1:
            raise ValueError("group table too small")
        _capi.need_experimental("DeviceReassembler.reassemble_groups")
        check(lib().e2sar_hip_reassemble_groups(
            self._h, C.c_void_p(packets.data_ptr()), stride, C.c_void_p(lens.data_ptr()), n,
            C.c_void_p(starts.data_ptr() if starts is not None else 0), n_groups if starts is not None else 0,
            int(now_ms), C.c_void_p(_stream_handle(stream))))

    def relay_plan(self, events: torch.Tensor, counts: torch.Tensor, first_record: int, max_events: int,
                   max_pld: int, lb_tick: int, entropy_base: int,
                   stream: Optional[torch.cuda.Stream] = None) -> None:
        """Completed records [first_record, +n) -> seg descriptors in `events` (uint8 device
        tensor of max_events * SEG_EVENT_BYTES) and counts[0:2] = (n, datagrams) (int32/uint32
        device tensor), without a host round trip (e2sar_hip_relay_plan)."""
        if events.numel() < max_events * SEG_EVENT_BYTES or counts.numel() < 2:
            raise ValueError("relay buffers too small")
        check(lib().e2sar_hip_relay_plan(
            self._h, first_record, max_events, max_pld, int(lb_tick), entropy_base & 0xFFFF,
            C.c_void_p(events.data_ptr()), C.c_void_p(counts.data_ptr()), C.c_void_p(_stream_handle(stream))))

    # ---- split form: classify (headers, table) then scatter (bytes), for pipelining ----
    @staticmethod
    def work_bytes(n: int) -> int:
        return int(lib().e2sar_hip_reas_work_bytes(int(n)))

    def alloc_work(self, n: int) -> torch.Tensor:
        """Device work buffer for one classified batch of up to n datagrams."""
        return torch.empty(self.work_bytes(n), dtype=torch.uint8, device=self.ctx.torch_device)

    def classify(self, packets: torch.Tensor, stride: int, lens: torch.Tensor, n: int, work: torch.Tensor,
                 now_ms: int = 0, stream: Optional[torch.cuda.Stream] = None) -> None:
        if n == 0:
            return
        if lens.numel() < n or packets.numel() < n * stride:
            raise ValueError("packet batch buffers too small")
        check(lib().e2sar_hip_reas_classify(
            self._h, C.c_void_p(packets.data_ptr()), stride, C.c_void_p(lens.data_ptr()), n, int(now_ms),
            C.c_void_p(work.data_ptr()), work.numel(), C.c_void_p(_stream_handle(stream))))

    def scatter(self, packets: torch.Tensor, stride: int, n: int, work: torch.Tensor,
                stream: Optional[torch.cuda.Stream] = None) -> None:
        if n == 0:
            return
        if packets.numel() < n * stride:
            raise ValueError("packet batch buffer too small")
        check(lib().e2sar_hip_reas_scatter(
            self._h, C.c_void_p(packets.data_ptr()), stride, n, C.c_void_p(work.data_ptr()), work.numel(),
            C.c_void_p(_stream_handle(stream))))

    def scatter_classify(self, stride: int, s_packets: torch.Tensor, s_n: int, s_work: torch.Tensor,
                         c_packets: torch.Tensor, c_lens: torch.Tensor, c_n: int, c_work: torch.Tensor,
                         now_ms: int = 0, stream: Optional[torch.cuda.Stream] = None) -> None:
        """One launch: scatter classified batch b while classifying batch b+1."""
        if s_n and s_packets.numel() < s_n * stride:
            raise ValueError("scatter batch buffer too small")
        if c_n and (c_lens.numel() < c_n or c_packets.numel() < c_n * stride):
            raise ValueError("classify batch buffers too small")
        check(lib().e2sar_hip_reas_scatter_classify(
            self._h, stride, C.c_void_p(s_packets.data_ptr()), s_n, C.c_void_p(s_work.data_ptr()), s_work.numel(),
            C.c_void_p(c_packets.data_ptr()), C.c_void_p(c_lens.data_ptr()), c_n, int(now_ms),
            C.c_void_p(c_work.data_ptr()), c_work.numel(), C.c_void_p(_stream_handle(stream))))

    def forget_stream(self, stream: torch.cuda.Stream) -> None:
        """Before the caller destroys `stream`, on which it launched through this reassembler:
        wait for it, stop tracking it and free its internal buffers
        (e2sar_hip_reas_forget_stream).  The stream must still be alive."""
        check(lib().e2sar_hip_reas_forget_stream(self._h, C.c_void_p(_stream_handle(stream))))

    def gc(self, now_ms: int, timeout_ms: int, stream: Optional[torch.cuda.Stream] = None) -> None:
        check(lib().e2sar_hip_reas_gc(self._h, int(now_ms), int(timeout_ms), C.c_void_p(_stream_handle(stream))))

    def poll(self) -> List[_capi.EventRec]:
        n = C.c_uint32()
        check(lib().e2sar_hip_reas_poll(self._h, self._evbuf, len(self._evbuf), C.byref(n)))
        out = []
        for k in range(n.value):
            r = _capi.EventRec()
            C.memmove(C.byref(r), C.byref(self._evbuf[k]), C.sizeof(r))
            out.append(r)
        return out

    def lost_poll(self) -> List[_capi.LostRec]:
        n = C.c_uint32()
        check(lib().e2sar_hip_reas_lost_poll(self._h, self._lostbuf, len(self._lostbuf), C.byref(n)))
        out = []
        for k in range(n.value):
            r = _capi.LostRec()
            C.memmove(C.byref(r), C.byref(self._lostbuf[k]), C.sizeof(r))
            out.append(r)
        return out

    def stats(self) -> _capi.ReasStats:
        s = _capi.ReasStats()
        check(lib().e2sar_hip_reas_get_stats(self._h, C.byref(s)))
        return s

    def recycle(self, force: bool = False, stream: Optional[torch.cuda.Stream] = None) -> None:
        check(lib().e2sar_hip_reas_recycle(self._h, 1 if force else 0, C.c_void_p(_stream_handle(stream))))

    def compact(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Move in-progress events to the alternate arena (see e2sar_hip_reas_compact)."""
        check(lib().e2sar_hip_reas_compact(self._h, C.c_void_p(_stream_handle(stream))))
        self.arena_ptr = int(lib().e2sar_hip_reas_arena(self._h) or 0)

    def reset_stats(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        check(lib().e2sar_hip_reas_reset_stats(self._h, C.c_void_p(_stream_handle(stream))))

    def event_bytes(self, rec: _capi.EventRec) -> bytes:
        """Copy one reassembled event to host memory."""
        buf = (C.c_uint8 * max(rec.bytes, 1))()
        if rec.bytes:
            check(lib().e2sar_hip_memcpy_d2h(self.ctx.handle, buf, C.c_void_p(self.arena_ptr + rec.arenaOffset),
                                             rec.bytes))
        return bytes(buf)[: rec.bytes]

    def arena_tensor(self) -> torch.Tensor:
        """Zero-copy uint8 view of the whole device arena."""
        return _device_view(self.arena_ptr, self.arena_bytes, self.ctx.torch_device)

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().e2sar_hip_reas_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _CudaArray:
    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {
            "shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 2, "strides": None,
        }


def _device_view(ptr: int, nbytes: int, device: torch.device) -> torch.Tensor:
    return torch.as_tensor(_CudaArray(ptr, nbytes), device=device)
