"""Probe: tests/test_gpu_dist.py's _nccl_worker run in this process (no spawn), with a plain
torch op after it, to localise the 'invalid device ordinal' of its regions_raw step."""
import os
import sys
import traceback

HERE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import test_gpu_dist as T


class Q:
    def put(self, x):
        print("result", x, flush=True)


try:
    T._nccl_worker(int(sys.argv[1]) if len(sys.argv) > 1 else 29536, Q())
except Exception:
    traceback.print_exc()
    print("RAISED", flush=True)
