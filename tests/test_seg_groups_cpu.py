"""e2sar_hip_seg_groups (host only): the reassembly group table that matches seg_kernel's
XCD stripes, against a restatement of the rule -- datagram (e, q) belongs to stripe
(e * unitsPerEvent + q * chunksPerSlot // unitChunks) // stripe; groups are the stripes in
order, at most 64 datagrams each, else no table.  Without a GPU the library knows no
residency to balance the stripe against, so the stripe is the unbalanced target (on a GPU,
tests/test_gpu_xcd_groups.py checks the balanced table by its results)."""
import ctypes as C

import pytest


def _experimental():
    try:
        from e2sar_amd import _capi
        return _capi.has_experimental()
    except ImportError:
        return False


pytestmark = pytest.mark.skipif(
    not _experimental(), reason="A/B-only form: make experimental; E2SAR_HIP_LIB=build/variants/lib_experimental.so")


def _geom(max_pk, stride):
    spc = stride // 16
    chunks = max_pk * spc
    U = 2 if chunks <= (1 << 18) else 4
    unit = 256 * U
    bpe = -(-chunks // unit)
    target = min(49, max(1, 9216 // spc))
    stripe = max(1, target * spc // unit)
    return spc, unit, bpe, stripe


def _restated(sizes, mp, stride):
    npk = [-(-s // mp) for s in sizes]
    spc, unit, bpe, stripe = _geom(max(npk), stride)  # the plan's maxPacketsPerEvent
    n_groups = -(-(bpe * len(sizes)) // stripe)
    members = [[] for _ in range(n_groups)]
    base = 0
    for e, n in enumerate(npk):
        for q in range(n):
            members[(e * bpe + q * spc // unit) // stripe].append(base + q)
        base += n
    starts = [0]
    for m in members:
        starts.append(starts[-1] + len(m))
    if any(len(m) > 64 for m in members):
        return 0, None
    return n_groups, starts


@pytest.mark.parametrize("mtu,sizes", [
    (1500, [1 << 20] * 205),
    (1500, [1, 15, 16, 17, 1435, 1436, 1437, 50000, 123457, 0, 1 << 20]),
    (9000, [1 << 20] * 64),
    (9000, [8 << 20] * 70),
    (9000, [8 << 20, 3 << 20, 8936 * 3 + 1]),
    (80, [1, 43, 44, 45, 1000, 4321]),
    (67, [5000, 31, 1]),
])
def test_seg_groups_matches_rule(mtu, sizes):
    from e2sar_amd import _capi
    L = _capi.lib()
    mp = L.e2sar_hip_max_pld_len(mtu, 0)
    stride = L.e2sar_hip_packet_stride(mp)
    arr = (_capi.SegEvent * len(sizes))()
    for k, s in enumerate(sizes):
        arr[k].bytes = s
    tot, mx = C.c_uint32(), C.c_uint32()
    assert L.e2sar_hip_seg_plan(arr, len(sizes), mp, C.byref(tot), C.byref(mx)) == 0
    cap = len(sizes) * (mx.value * (stride // 16) // 512 + 2) + 2
    starts = (C.c_uint32 * cap)()
    ng = C.c_uint32()
    assert L.e2sar_hip_seg_groups(arr, len(sizes), mx.value, mp, stride, starts, cap, C.byref(ng)) == 0
    want_ng, want = _restated(sizes, mp, stride)
    assert ng.value == want_ng
    if want_ng:
        assert list(starts[: want_ng + 1]) == want
        assert want[-1] == tot.value
        assert max(b - a for a, b in zip(want, want[1:])) <= 64


def test_seg_groups_small_cap_returns_zero():
    from e2sar_amd import _capi
    L = _capi.lib()
    mp = L.e2sar_hip_max_pld_len(1500, 0)
    stride = L.e2sar_hip_packet_stride(mp)
    arr = (_capi.SegEvent * 4)()
    for k in range(4):
        arr[k].bytes = 1 << 20
    tot, mx = C.c_uint32(), C.c_uint32()
    assert L.e2sar_hip_seg_plan(arr, 4, mp, C.byref(tot), C.byref(mx)) == 0
    starts = (C.c_uint32 * 3)()
    ng = C.c_uint32(7)
    assert L.e2sar_hip_seg_groups(arr, 4, mx.value, mp, stride, starts, 3, C.byref(ng)) == 0
    assert ng.value == 0
