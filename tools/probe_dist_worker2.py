"""Probe: the RCCL world-1 regions_raw step of tests/test_gpu_dist.py, alone or after the
pipeline_all mode (argv[1]: none | pipeline_all | pipeline_all_gc), each with a torch op after."""
import gc
import os
import sys
import traceback

HERE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29537")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
import torch
import torch.distributed as dist

dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
import test_gpu_dist as T
from e2sar_amd import sar
from e2sar_amd.dist import RegionRouter

pre = sys.argv[1] if len(sys.argv) > 1 else "none"
if pre.startswith("pipeline_all"):
    print("pre", T._spread_rank(0, 1, "pipeline_all", corrupt=False)[1], flush=True)
    if pre.endswith("gc"):
        gc.collect()
        torch.cuda.synchronize()
try:
    stride, n = 1472, 300
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    spk = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device="cuda", generator=g)
    ctx = sar.Context(0)
    rr = RegionRouter(ctx, stride, 2 * n, n, 1, 0, with_lb_header=True, foreign_only=False)
    rr.reset()
    spk2 = spk.clone()
    for k in range(n):
        spk2[k * stride + 16] = 0x10
        spk2[k * stride + 17] = 0
    sln2 = torch.full((n,), stride, dtype=torch.int32, device="cuda")
    rr.route(spk2, sln2, n // 2)
    rr.route(spk2[(n // 2) * stride:], sln2[n // 2:], n - n // 2)
    print("routed", flush=True)
    torch.cuda.synchronize()
    print("running", rr.running.tolist(), flush=True)
    rpk2, rln2, nr2 = rr.exchange()
    torch.cuda.synchronize()
    print("exchanged", nr2, flush=True)
    print("equal", bool(torch.equal(rln2[:n], sln2)), flush=True)
except Exception:
    traceback.print_exc()
    print("RAISED", flush=True)
dist.destroy_process_group()
