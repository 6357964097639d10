"""Probe: tests/test_gpu_dist.py's RCCL world-1 worker, one mode at a time, with a plain
torch op after each to find which mode leaves the process in a bad state."""
import os
import sys

HERE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29535")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
import torch
import torch.distributed as dist

dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
import test_gpu_dist as T

x = torch.full((8,), 3, dtype=torch.int32, device="cuda")
for mode in sys.argv[1:]:
    try:
        r = T._spread_rank(0, 1, mode, corrupt=False)
        print(mode, "ok" if r[1] else "MISMATCH", r[2:], flush=True)
    except Exception as e:
        print(mode, "RAISED", type(e).__name__, str(e)[:300], flush=True)
    try:
        torch.cuda.synchronize()
        print("  equal after", mode, bool(torch.equal(x, x.clone())), flush=True)
    except Exception as e:
        print("  equal after", mode, "FAILED", type(e).__name__, str(e)[:200], flush=True)
        break
dist.destroy_process_group()
