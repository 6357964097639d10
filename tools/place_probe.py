"""Placement probe for config 3's reassembly (70 x 8 MiB at MTU 9000, 65,730 datagrams,
590 MB of slots per launch, more than the Infinity Cache): does the launch time depend on
where the datagram buffer sits relative to the event arena?

For each offset of the datagram buffer (inside one allocation, so the virtual-to-physical
mapping is the same for every trial) and each shift of the arena's first event (a dummy
event reassembled first takes that much of the arena), segment the batch, reassemble it
(reassemble_batch: classify + scatter inside) and time both with HIP events; the arena is
recycled between trials.  Prints one JSON line per (offset, shift).
Usage: python tools/place_probe.py [--trials 3]
"""
import argparse
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from e2sar_amd import sar  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--events", type=int, default=70)
    ap.add_argument("--event-bytes", type=int, default=8 << 20)
    ap.add_argument("--mtu", type=int, default=9000)
    ap.add_argument("--offsets-mib", default="0,0.0625,0.25,1,2,3,4,6,8,16,32")
    ap.add_argument("--shifts-mib", default="0,1,4")
    ap.add_argument("--copy", action="store_true",
                    help="also time a plain copy of the just-written datagram buffer (copy_spans, the floor)")
    ap.add_argument("--split", action="store_true", help="also time classify and scatter (streaming loads) apart")
    ap.add_argument("--pk-lib", action="store_true",
                    help="allocate the datagram buffer with e2sar_hip_device_alloc instead of torch")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = sar.Context(0)
    E, B = a.events, a.event_bytes
    src = torch.empty(E * B, dtype=torch.uint8, device=dev)
    src.random_(0, 256)
    seg = sar.DeviceSegmenter(ctx, mtu=a.mtu)
    plan = seg.plan([(src.data_ptr() + k * B, B, k, 4321, 1 + k, (1 << 48) + k) for k in range(E)])
    n, stride = plan.total_packets, seg.stride
    offs = [int(float(x) * (1 << 20)) // 16 * 16 for x in a.offsets_mib.split(",")]
    shifts = [int(float(x) * (1 << 20)) for x in a.shifts_mib.split(",")]
    if a.pk_lib:
        import ctypes as C
        from e2sar_amd._capi import check, lib
        nb = n * stride + max(offs) + 16
        ptr = C.c_void_p()
        check(lib().e2sar_hip_device_alloc(ctx.handle, C.c_size_t(nb), C.byref(ptr)))
        pkall = sar._device_view(ptr.value, nb, dev)
    else:
        pkall = torch.empty(n * stride + max(offs) + 16, dtype=torch.uint8, device=dev)
    ln = torch.empty(n, dtype=torch.int32, device=dev)
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=4096, queue_capacity=4096,
                              arena_bytes=E * (B + 256) + max(shifts) + (64 << 20))
    dsrc = torch.empty(max(max(shifts), 1), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for o in offs:
        pk = pkall[o:o + n * stride]
        for sh in shifts:
            seg_us, reas_us = [], []
            for t in range(a.trials + 1):
                R.recycle(force=True)
                if sh:
                    # one dummy event of sh bytes reassembled first: the batch's events start sh further in
                    dplan = seg.plan([(dsrc.data_ptr(), sh, 1 << 40, 4321, 1, 1)])
                    dpk, dln = seg.alloc_packets(dplan.total_packets)
                    seg.segment(dplan, dpk, dln)
                    R.reassemble(dpk, stride, dln, dplan.total_packets)
                ev[0].record(s)
                seg.segment(plan, pk, ln)
                ev[1].record(s)
                R.reassemble(pk, stride, ln, n)
                ev[2].record(s)
                torch.cuda.synchronize()
                R.poll()
                if t:
                    seg_us.append(round(ev[0].elapsed_time(ev[1]) * 1000, 1))
                    reas_us.append(round(ev[1].elapsed_time(ev[2]) * 1000, 1))
            cls_us, sc_us = [], []
            if a.split:
                work = R.alloc_work(n)
                R.set_cold(True)
                for t in range(a.trials + 1):
                    R.recycle(force=True)
                    seg.segment(plan, pk, ln)
                    ev[0].record(s)
                    R.classify(pk, stride, ln, n, work)
                    ev[1].record(s)
                    R.scatter(pk, stride, n, work)
                    ev[2].record(s)
                    torch.cuda.synchronize()
                    R.poll()
                    if t:
                        cls_us.append(round(ev[0].elapsed_time(ev[1]) * 1000, 1))
                        sc_us.append(round(ev[1].elapsed_time(ev[2]) * 1000, 1))
                R.set_cold(False)
                del work
            copy_us = []
            if a.copy:
                dst = torch.empty(n * stride, dtype=torch.uint8, device=dev)
                for t in range(a.trials + 1):
                    seg.segment(plan, pk, ln)
                    ev[1].record(s)
                    ctx.copy_spans([(pk.data_ptr(), dst.data_ptr(), n * stride)])
                    ev[2].record(s)
                    torch.cuda.synchronize()
                    if t:
                        copy_us.append(round(ev[1].elapsed_time(ev[2]) * 1000, 1))
                del dst
            st = R.stats()
            print(json.dumps({"pk_off": o, "arena_shift": sh, "pk_addr_mod_2M": (pk.data_ptr() % (2 << 20)),
                              "arena_rel": (R.arena_ptr + sh - pk.data_ptr()),
                              "seg_us": seg_us, "reas_us": reas_us, "copy_us": copy_us, "classify_us": cls_us, "scatter_us": sc_us, "errflags": int(st.errorFlags)}), flush=True)


if __name__ == "__main__":
    main()
