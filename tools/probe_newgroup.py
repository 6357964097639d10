"""Probe: a second RCCL communicator (dist.new_group) beside the default one, world 1, each
collective from a stream of its own -- the SpreadPipeline count group's shape.
Usage: python tools/probe_newgroup.py VARIANT   (plain | devid | both)"""
import os
import sys

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
import torch
import torch.distributed as dist

v = sys.argv[1] if len(sys.argv) > 1 else "plain"
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
kw = {"device_id": dev} if v in ("devid", "both") else {}
try:
    g2 = dist.new_group(ranks=[0], backend="nccl", **kw)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.arange(4, dtype=torch.int32, device=dev)
    out = torch.empty(4, dtype=torch.int32, device=dev)
    with torch.cuda.stream(s2):
        dist.all_gather_into_tensor(out, a, group=g2)
    with torch.cuda.stream(s1):
        x = torch.randint(0, 255, (1 << 20,), dtype=torch.uint8, device=dev)
        y = torch.empty_like(x)
        dist.all_to_all([y], [x])
    torch.cuda.synchronize()
    print(v, "ok", out.tolist(), bool(torch.equal(x, y)), flush=True)
except Exception as e:                      # report, do not crash the session
    print(v, "FAILED", type(e).__name__, str(e)[:300], flush=True)
dist.destroy_process_group()
