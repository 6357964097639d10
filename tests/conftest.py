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
