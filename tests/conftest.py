import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def hip():
    """Device context for GPU tests; fails loudly if the HIP library is missing."""
    import torch
    from e2sar_amd import sar

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no GPU is visible")
    ctx = sar.Context(0)
    yield ctx
    ctx.sync()


def _size(x, cap=1 << 16):
    """Rough byte size of an assertion operand (stops counting at cap)."""
    if isinstance(x, (bytes, bytearray, str)):
        return len(x)
    if isinstance(x, dict):
        x = list(x.items())
    if isinstance(x, (list, tuple, set)):
        n = 0
        for v in x:
            n += _size(v, cap)
            if n >= cap:
                break
        return n
    return 8


def pytest_assertrepr_compare(op, left, right):
    """Event payloads are megabytes: pytest's default diff of two such operands runs for
    minutes (difflib), long enough to look like a hung GPU test.  Summarise instead."""
    if _size(left) + _size(right) < (1 << 16):
        return None
    out = [f"large operands ({type(left).__name__} {op} {type(right).__name__}) differ"]
    if isinstance(left, dict) and isinstance(right, dict):
        out.append(f"keys only left: {sorted(set(left) - set(right))[:8]}; only right: {sorted(set(right) - set(left))[:8]}")
        out.append(f"keys with different values: {[k for k in left if k in right and left[k] != right[k]][:8]}")
    elif isinstance(left, (list, tuple)) and isinstance(right, (list, tuple)):
        diff = [i for i, (a, b) in enumerate(zip(left, right)) if a != b]
        out.append(f"lengths {len(left)} / {len(right)}; first differing items {diff[:8]}")
    elif isinstance(left, (bytes, bytearray)) and isinstance(right, (bytes, bytearray)):
        diff = [i for i, (a, b) in enumerate(zip(left, right)) if a != b]
        out.append(f"lengths {len(left)} / {len(right)}; {len(diff)} differing bytes, first at {diff[:8]}")
    return out
