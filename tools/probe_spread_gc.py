"""Probe: build a SpreadPipeline (route-all form, RCCL world 1), land a few batches, drop it,
gc, then a plain torch op.  argv[1]: newgroup (count group created by the pipeline) |
world (count group = the default group) | keepref (new group, pipeline kept alive)."""
import gc
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29538")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
import torch
import torch.distributed as dist

dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
from e2sar_amd import sar
from e2sar_amd.dist import SpreadPipeline

v = sys.argv[1] if len(sys.argv) > 1 else "newgroup"
keep = []


def run():
    ctx = sar.Context(0)
    seg = sar.DeviceSegmenter(ctx, mtu=1500)
    src = torch.randint(0, 256, (8, 100_000), dtype=torch.uint8, device="cuda")
    plan = seg.plan([(src[i].data_ptr(), 100_000, i, 4321, 1 + i, 1 + i) for i in range(8)])
    pk, ln = seg.alloc_packets(plan.total_packets)
    seg.segment(plan, pk, ln)
    n = plan.total_packets
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=256, arena_bytes=1 << 24)
    kw = {"count_group": dist.group.WORLD} if v == "world" else {}
    pipe = SpreadPipeline(ctx, R, seg.stride, n, 1, 0, in_place=False, **kw)
    R.set_cold(True)
    pipe.begin_step()
    for a in range(0, n, n // 4 + 1):
        b = min(n, a + n // 4 + 1)
        pipe.land(pk[a * seg.stride:], ln[a:], b - a)
    pipe.flush()
    torch.cuda.synchronize()
    recs = R.poll()
    if v == "keepref":
        keep.append((pipe, R, ctx))
    return len(recs)


try:
    print("events", run(), flush=True)
    gc.collect()
    x = torch.full((8,), 3, dtype=torch.int32, device="cuda")
    print("torch op after gc", bool(torch.equal(x, x.clone())), flush=True)
except Exception:
    traceback.print_exc()
    print("RAISED", flush=True)
dist.destroy_process_group()
