"""Deterministic synthetic inputs shared by tests, fixtures and bench.py.

Payload bytes come from splitmix64 seeded with 0xE25A2 + event index,
so misplaced bytes are detectable.  Event metadata follows e2sar_perf's sender
(bin/e2sar_perf.cpp:175,396): eventNum = i, dataId = 4321, plus a nonzero injected
entropy and LB tick (the reference draws both at random, e2sarDPSegmenter.cpp:707-728).
"""
from __future__ import annotations

import numpy as np

SEED = 0xE25A2
DATA_ID = 4321
M64 = (1 << 64) - 1


def splitmix64_bytes(seed: int, nbytes: int) -> np.ndarray:
    n = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        x = (np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
             + np.uint64(seed & M64))
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:nbytes].copy()


def event_bytes(i: int, nbytes: int) -> np.ndarray:
    return splitmix64_bytes(SEED + i, nbytes)


def entropy(i: int) -> int:
    return 1 + (i * 0x9E37) % 65535


def lb_tick(i: int) -> int:
    return 0x0001_0000_0000_0000 + i
