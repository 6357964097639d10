#!/usr/bin/env python3
"""Split-reassembly stress on the GPU: the bench workload, step by step, synchronising and
checking stats/errorFlags after every step (eager), then graph replays one at a time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from e2sar_amd import sar
    mode = sys.argv[1] if len(sys.argv) > 1 else "split"
    dev = torch.device("cuda", 0)
    ctx = sar.Context(0)
    B, E, BE = 1 << 20, 1024, 128
    seg = sar.DeviceSegmenter(ctx, mtu=1500)
    stride = seg.stride
    evs = (B + 255) // 256 * 256
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    src = torch.randint(0, 256, (E, evs), dtype=torch.uint8, device=dev, generator=g)
    plans = [seg.plan([(src[i].data_ptr(), B, i, 4321, 1 + i, (1 << 48) + i) for i in range(b0, b0 + BE)])
             for b0 in range(0, E, BE)]
    npk = plans[0].total_packets
    pk, ln = seg.alloc_packets(npk)
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=4096, queue_capacity=E + 64,
                              lost_capacity=1024, arena_bytes=E * evs + 4096)
    work = R.alloc_work(npk)

    def step():
        R.recycle(force=True)
        for p in plans:
            seg.segment(p, pk, ln)
            if mode == "fused":
                R.reassemble(pk, stride, ln, p.total_packets)
            else:
                R.classify(pk, stride, ln, p.total_packets, work)
                R.scatter(pk, stride, p.total_packets, work)

    def check(tag):
        torch.cuda.synchronize()
        st = R.stats()
        hdr = work[:4].view(torch.int32).item() if mode != "fused" else -1
        print(tag, "nFin", hdr, "eventSuccess", st.eventSuccess, "inProgress", st.inProgress, "errorFlags", st.errorFlags,
              "dataErr", st.dataErrCnt, "bad", st.badHeaderDiscards, flush=True)
        R.reset_stats()

    for k in range(25):
        step()
        check(f"eager {k}")
    graph = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):
        step()
    torch.cuda.synchronize()
    with torch.cuda.graph(graph, stream=cap):
        step()
    for k in range(25):
        graph.replay()
        check(f"replay {k}")
    t0 = time.time()
    for k in range(20):
        graph.replay()
    check(f"replay x20 {time.time() - t0:.4f}s")


if __name__ == "__main__":
    main()
