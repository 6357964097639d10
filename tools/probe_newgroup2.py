"""Probe: does creating and using a second RCCL communicator (dist.new_group) disturb later
plain torch ops in the process (HIP 'invalid device ordinal' seen in test_gpu_dist.py)?"""
import gc
import os
import sys

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29534")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
import torch
import torch.distributed as dist

v = sys.argv[1] if len(sys.argv) > 1 else "devid"
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)


def use_group():
    kw = {"device_id": dev} if v == "devid" else {}
    g2 = dist.new_group(ranks=[0], backend="nccl", **kw)
    s2 = torch.cuda.Stream(dev)
    a = torch.arange(4, dtype=torch.int32, device=dev)
    out = torch.empty(4, dtype=torch.int32, device=dev)
    with torch.cuda.stream(s2):
        dist.all_gather_into_tensor(out, a, group=g2)
    torch.cuda.synchronize()
    return out.tolist()


def step(name, fn):
    try:
        print(name, "->", fn(), "current_device", torch.cuda.current_device(), flush=True)
    except Exception as e:
        print(name, "FAILED", type(e).__name__, str(e)[:200], flush=True)


x = torch.full((8,), 3, dtype=torch.int32, device="cuda")
step("equal before", lambda: bool(torch.equal(x, x.clone())))
step("group", use_group)
step("equal after", lambda: bool(torch.equal(x, x.clone())))
gc.collect()
step("equal after gc", lambda: bool(torch.equal(x, x.clone())))
step("full+equal", lambda: bool(torch.equal(torch.full((8,), 3, dtype=torch.int32, device="cuda"), x)))
dist.destroy_process_group()
