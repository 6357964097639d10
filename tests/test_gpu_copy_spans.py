"""e2sar_hip_copy_spans (the façade's gather of completed events, and the bench's HBM copy
calibration): every byte of every span lands, for any size and alignment, device to
device and device to pinned host memory, more spans than one launch takes."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 15, 16, 17, 255, 16383, 16384, 16385, 65536 + 7, (1 << 20) + 3]


def test_copy_spans_device_to_device(hip):
    import torch
    from e2sar_amd import sar  # noqa: F401
    rng = np.random.default_rng(11)
    spans, checks = [], []
    total = sum(SIZES) * 2 + 64 * 4096
    src = torch.from_numpy(rng.integers(0, 256, total, dtype=np.uint8)).to(hip.torch_device)
    dst = torch.zeros(sum(SIZES) * 7 + 77 * 8 + 4096, dtype=torch.uint8, device=hip.torch_device)
    so = do = 0
    for k, n in enumerate(SIZES * 7):                  # 77 spans: two launches
        sa, da = so + (k % 3) * 4, do + (k % 5)          # aligned and misaligned both sides
        spans.append((src.data_ptr() + sa, dst.data_ptr() + da, n))
        checks.append((sa, da, n))
        so = (sa + n + 255) // 256 * 256 % (total - (1 << 21))
        do = da + n + 1
    hip.copy_spans(spans)
    torch.cuda.synchronize()
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()
    for sa, da, n in checks:
        assert np.array_equal(hd[da:da + n], hs[sa:sa + n]), (sa, da, n)


def test_copy_spans_device_to_pinned_host(hip):
    import torch
    from e2sar_amd._capi import check, lib
    n = (3 << 20) + 5
    src = torch.from_numpy(np.random.default_rng(12).integers(0, 256, n, dtype=np.uint8)).to(hip.torch_device)
    p = C.c_void_p()
    check(lib().e2sar_hip_host_alloc(n, C.byref(p)))
    try:
        hip.copy_spans([(src.data_ptr(), p.value, n)])
        torch.cuda.synchronize()
        got = np.ctypeslib.as_array((C.c_uint8 * n).from_address(p.value))
        assert np.array_equal(got, src.cpu().numpy())
    finally:
        lib().e2sar_hip_host_free(p)
