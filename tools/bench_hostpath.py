#!/usr/bin/env python3
"""Config 5: host <-> device SAR with pinned buffers (DESIGN.md number, not bench.py's value).

Receive direction: pinned host datagram batches (what recvmmsg fills) -> H2D -> reas_kernel
-> completed events D2H into pinned host memory (what getEvent hands out).
Send direction: pinned host events -> H2D -> seg_kernel -> datagrams D2H into pinned host
memory (what sendmmsg drains).  Relay (BASELINE config 5): pinned datagram batches -> H2D ->
reas_kernel -> relay_plan_kernel + seg_kernel on the reassembled events (no host round trip)
-> datagrams D2H; the host learns each batch's datagram count from a 8-byte D2H one batch
behind, so the GPU is never idle waiting for it.  Each direction runs on two streams -- H2D copy + kernel on
one, D2H copy on the other -- over --slots rotating buffer sets, so the whole process
uses four streams (GPU_MAX_HW_QUEUES is 4: more streams than hardware queues share
queues and serialise).  "both" runs the two directions at once (PCIe is full duplex).
Prints one JSON line: payload GiB/s per direction and both-at-once, plus PCIe-only rates.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# D2H copies into pinned memory run as blit kernels on the compute queues.  With the
# default 4 hardware queues per process, the four pipeline streams + the default stream
# share queues, and a D2H blit queued behind the next batch's kernel serialises the
# pipeline (send ran at half the PCIe rate).  8 queues give every stream its own.
os.environ["GPU_MAX_HW_QUEUES"] = "8"   # the box exports 4
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mtu", type=int, default=1500)
    ap.add_argument("--event-bytes", type=int, default=1 << 20)
    ap.add_argument("--batch-events", type=int, default=32)
    ap.add_argument("--batches", type=int, default=64)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--only", choices=["recv", "send", "both", "relay"], default=None,
                    help="time one mode only (for tracing)")
    ap.add_argument("--copy", choices=["dma", "kernel-d2h", "kernel"], default="dma",
                    help="dma: hipMemcpyAsync for both directions; kernel-d2h: device->host copies by "
                         "e2sar_hip_copy_spans (the GPU stores into pinned host memory); kernel: both "
                         "directions by copy_spans (the GPU loads from / stores to pinned host memory)")
    args = ap.parse_args()

    import torch
    from e2sar_amd import sar

    dev = torch.device("cuda", 0)
    ctx = sar.Context(0)
    B, BE = args.event_bytes, args.batch_events
    seg = sar.DeviceSegmenter(ctx, mtu=args.mtu)
    stride, npk = seg.stride, sar.num_packets(args.event_bytes, seg.max_pld)
    bpk = BE * npk                      # datagrams per batch
    ev_stride = (B + 255) // 256 * 256

    # ---------------- inputs: pinned host events and pinned host datagram batches ----------------
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    dev_events = torch.randint(0, 256, (BE, ev_stride), dtype=torch.uint8, device=dev, generator=g)
    S = args.slots
    h_events = [torch.empty((BE, ev_stride), dtype=torch.uint8).pin_memory() for _ in range(S)]
    for h in h_events:
        h.copy_(dev_events)
    # build the datagram batch once on the device (any event numbers; each batch reuses them)
    plan0 = seg.plan([(dev_events[i].data_ptr(), B, i, 4321, 1 + i, 7 + i) for i in range(BE)])
    pk0, ln0 = seg.alloc_packets(bpk)
    seg.segment(plan0, pk0, ln0)
    torch.cuda.synchronize()
    h_pk = [torch.empty(bpk * stride, dtype=torch.uint8).pin_memory() for _ in range(S)]
    h_ln = [torch.empty(bpk, dtype=torch.int32).pin_memory() for _ in range(S)]
    for a, b in zip(h_pk, h_ln):
        a.copy_(pk0[: bpk * stride])
        b.copy_(ln0[:bpk])
    h_out_events = [torch.empty((BE, ev_stride), dtype=torch.uint8).pin_memory() for _ in range(S)]
    h_out_pk = [torch.empty(bpk * stride, dtype=torch.uint8).pin_memory() for _ in range(S)]

    # ---------------- device buffers ----------------
    d_pk = [torch.empty(bpk * stride, dtype=torch.uint8, device=dev) for _ in range(S)]
    d_ln = [torch.empty(bpk, dtype=torch.int32, device=dev) for _ in range(S)]
    d_ev = [torch.empty((BE, ev_stride), dtype=torch.uint8, device=dev) for _ in range(S)]
    d_spk = [seg.alloc_packets(bpk) for _ in range(S)]
    plans = [seg.plan([(d_ev[s][i].data_ptr(), B, i, 4321, 1 + i, 7 + i) for i in range(BE)]) for s in range(S)]
    # one reassembler per slot: a slot's arena is recycled only after its previous D2H finished
    R = [sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=max(64, 1 << (2 * BE).bit_length()),
                               queue_capacity=4 * BE, arena_bytes=BE * ev_stride + 4096) for _ in range(S)]
    arena_views = [r.arena_tensor()[: BE * ev_stride] for r in R]   # built once (CAI import may sync)
    rs = [torch.cuda.Stream() for _ in range(2)]      # recv: H2D + kernel, D2H
    ss = [torch.cuda.Stream() for _ in range(2)]      # send: H2D + kernel, D2H

    def h2d(dst, src):
        """host -> device copy on the current stream (DMA or a copy_spans kernel)."""
        if args.copy == "kernel":
            ctx.copy_spans([(src.data_ptr(), dst.data_ptr(), src.numel() * src.element_size())],
                           stream=torch.cuda.current_stream())
        else:
            dst.copy_(src, non_blocking=True)

    def d2h(dst, src):
        if args.copy in ("kernel", "kernel-d2h"):
            ctx.copy_spans([(src.data_ptr(), dst.data_ptr(), src.numel() * src.element_size())],
                           stream=torch.cuda.current_stream())
        else:
            dst.copy_(src, non_blocking=True)

    def recv_batch(k, ev_done):
        s = k % S
        with torch.cuda.stream(rs[0]):
            if ev_done[s] is not None:
                rs[0].wait_event(ev_done[s])
            h2d(d_pk[s], h_pk[s])
            h2d(d_ln[s], h_ln[s])
            R[s].recycle(force=True, stream=rs[0])    # events of this batch fill arena[0, BE*ev_stride)
            R[s].reassemble(d_pk[s], stride, d_ln[s], bpk, stream=rs[0])
            e1 = torch.cuda.Event()
            e1.record(rs[0])
        rs[1].wait_event(e1)
        with torch.cuda.stream(rs[1]):
            # the batch's events fill the recycled arena contiguously (256-B aligned buffers)
            d2h(h_out_events[s].view(-1), arena_views[s])
            e2 = torch.cuda.Event()
            e2.record(rs[1])
        ev_done[s] = e2

    def send_batch(k, ev_done):
        s = k % S
        with torch.cuda.stream(ss[0]):
            if ev_done[s] is not None:
                ss[0].wait_event(ev_done[s])
            h2d(d_ev[s], h_events[s])
            seg.segment(plans[s], d_spk[s][0], d_spk[s][1], stream=ss[0])
            e1 = torch.cuda.Event()
            e1.record(ss[0])
        ss[1].wait_event(e1)
        with torch.cuda.stream(ss[1]):
            d2h(h_out_pk[s], d_spk[s][0][: bpk * stride])
            e2 = torch.cuda.Event()
            e2.record(ss[1])
        ev_done[s] = e2

    # relay: datagrams in, the reassembled events segmented again on the device, datagrams out
    relay_desc = [torch.zeros(BE * sar.SEG_EVENT_BYTES, dtype=torch.uint8, device=dev) for _ in range(S)]
    relay_cnt = [torch.zeros(2, dtype=torch.int32, device=dev) for _ in range(S)]
    relay_hcnt = [torch.zeros(2, dtype=torch.int32).pin_memory() for _ in range(S)]

    def relay_front(k, ev_done, ev_cnt):
        s = k % S
        with torch.cuda.stream(rs[0]):
            if ev_done[s] is not None:
                rs[0].wait_event(ev_done[s])
            h2d(d_pk[s], h_pk[s])
            h2d(d_ln[s], h_ln[s])
            R[s].recycle(force=True, stream=rs[0])
            R[s].reassemble(d_pk[s], stride, d_ln[s], bpk, stream=rs[0])
            R[s].relay_plan(relay_desc[s], relay_cnt[s], 0, BE, seg.max_pld, 7 + k, 1 + k, stream=rs[0])
            seg.segment_device(relay_desc[s], relay_cnt[s], BE, npk, d_spk[s][0], d_spk[s][1], stream=rs[0])
            relay_hcnt[s].copy_(relay_cnt[s], non_blocking=True)
            e1 = torch.cuda.Event()
            e1.record(rs[0])
        ev_cnt[s] = e1

    def relay_back(k, ev_done, ev_cnt):
        s = k % S
        ev_cnt[s].synchronize()                  # the batch's datagram count, one batch behind
        total = int(relay_hcnt[s][1])
        rs[1].wait_event(ev_cnt[s])
        with torch.cuda.stream(rs[1]):
            d2h(h_out_pk[s][: total * stride], d_spk[s][0][: total * stride])
            e2 = torch.cuda.Event()
            e2.record(rs[1])
        ev_done[s] = e2
        return total

    def run(mode):
        best = 0.0
        for _ in range(args.iters):
            torch.cuda.synchronize()
            rd, sd, rc = [None] * S, [None] * S, [None] * S
            t0 = time.perf_counter()
            for k in range(args.batches):
                if mode == "relay":
                    relay_front(k, rd, rc)
                    if k:
                        relay_back(k - 1, rd, rc)
                    continue
                if mode in ("recv", "both"):
                    recv_batch(k, rd)
                if mode in ("send", "both"):
                    send_batch(k, sd)
            if mode == "relay":
                relay_back(args.batches - 1, rd, rc)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = max(best, args.batches * BE * B / dt / 2**30)
        return best

    # correctness of the recv direction: the reassembled batch equals the source events
    rd = [None] * S
    recv_batch(0, rd)
    torch.cuda.synchronize()
    recs = R[0].poll()
    assert len(recs) == BE, len(recs)
    arena = R[0].arena_tensor()
    for r in recs:
        assert torch.equal(arena[r.arenaOffset: r.arenaOffset + B], dev_events[r.eventNum, :B])

    res = {"config": f"host path: {BE} x {B} B events per batch, MTU {args.mtu}, pinned buffers, "
                     f"2 streams per direction (H2D+kernel, D2H), {S} rotating buffer sets, copies: {args.copy}"}
    if args.only:
        res[args.only + "_GiBps"] = round(run(args.only), 2)
        print(json.dumps(res), flush=True)
        return
    # correctness of the relay: one batch through, the re-sent datagrams carry every event
    rd, rc = [None] * S, [None] * S
    relay_front(0, rd, rc)
    total = relay_back(0, rd, rc)
    torch.cuda.synchronize()
    assert total == bpk, (total, bpk)
    res.update({"recv_GiBps": round(run("recv"), 2), "send_GiBps": round(run("send"), 2),
                "both_GiBps_each_direction": round(run("both"), 2), "relay_GiBps": round(run("relay"), 2)})
    # PCIe alone: the same copies without kernels
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.batches):
        d_pk[k % S].copy_(h_pk[k % S], non_blocking=True)
    torch.cuda.synchronize()
    res["pcie_h2d_GBps"] = round(args.batches * bpk * stride / (time.perf_counter() - t0) / 1e9, 1)
    t0 = time.perf_counter()
    for k in range(args.batches):
        h_out_pk[k % S].copy_(d_spk[k % S][0][: bpk * stride], non_blocking=True)
    torch.cuda.synchronize()
    res["pcie_d2h_GBps"] = round(args.batches * bpk * stride / (time.perf_counter() - t0) / 1e9, 1)
    # both directions at once, copies only, one stream per direction
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.batches):
        with torch.cuda.stream(rs[0]):
            d_pk[k % S].copy_(h_pk[k % S], non_blocking=True)
        with torch.cuda.stream(rs[1]):
            h_out_pk[k % S].copy_(d_spk[k % S][0][: bpk * stride], non_blocking=True)
    torch.cuda.synchronize()
    res["pcie_bidir_GBps_each"] = round(args.batches * bpk * stride / (time.perf_counter() - t0) / 1e9, 1)
    # the same with copy_spans kernels (the GPU's own loads / stores across PCIe)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.batches):
        with torch.cuda.stream(rs[0]):
            ctx.copy_spans([(h_pk[k % S].data_ptr(), d_pk[k % S].data_ptr(), bpk * stride)], stream=rs[0])
        with torch.cuda.stream(rs[1]):
            ctx.copy_spans([(d_spk[k % S][0].data_ptr(), h_out_pk[k % S].data_ptr(), bpk * stride)], stream=rs[1])
    torch.cuda.synchronize()
    res["pcie_bidir_kernel_GBps_each"] = round(args.batches * bpk * stride / (time.perf_counter() - t0) / 1e9, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
