"""Reassembly over the XCD-stripe group table (e2sar_hip_seg_groups +
e2sar_hip_reassemble_groups) against the uniform-group path and the source bytes.

Bar: every event completes with its source bytes and numFragments, and every counter
equals e2sar_hip_reassemble_batch's on the same datagrams -- over full-size and ragged
batches, misaligned events, MTU 80 / 1500 / 9000, LB v2 and v3, and back-to-back batches
into one reassembler; a batch without stripes (nGroups 0) falls back to the uniform
groups.  The receive body is e2sarDPReassembler.cpp:335-427 either way.
"""
import numpy as np
import pytest

def _experimental():
    try:
        from e2sar_amd import _capi
        return _capi.has_experimental()
    except ImportError:
        return False


pytestmark = [pytest.mark.gpu, pytest.mark.skipif(
    not _experimental(), reason="A/B-only form: make experimental; E2SAR_HIP_LIB=build/variants/lib_experimental.so")]

STATS = ("eventSuccess", "totalPackets", "totalBytes", "badHeaderDiscards", "dataErrCnt", "inProgress")


def _rng_bytes(seed, n):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


def _run(ctx, sizes, mtu, ver, use_groups, misalign=False, seed=0, launches=2):
    import torch
    from e2sar_amd import sar
    evs = [_rng_bytes(seed * 1000 + k, s) for k, s in enumerate(sizes)]
    offs, cur = [], 0
    for k, s in enumerate(sizes):
        cur = (cur + 255) // 256 * 256 + (k % 4 if misalign else 0)
        offs.append(cur)
        cur += s
    host = np.zeros(max(cur, 1), np.uint8)
    for e, o in zip(evs, offs):
        host[o:o + len(e)] = e
    dsrc = torch.from_numpy(host).to(ctx.torch_device)
    seg = sar.DeviceSegmenter(ctx, mtu=mtu, lb_hdr_version=ver)
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=2048, queue_capacity=2048,
                              arena_bytes=max(64 << 20, launches * (sum(sizes) + 256 * len(sizes))))
    out, ngs = [], []
    for L in range(launches):
        plan = seg.plan([(dsrc.data_ptr() + o, len(e), 1000 * L + k, 7, k, (1 << 40) + k)
                         for k, (e, o) in enumerate(zip(evs, offs))])
        pk, ln = seg.alloc_packets(plan.total_packets)
        seg.segment(plan, pk, ln)
        if use_groups:
            starts, ng = seg.groups(plan)
            ngs.append(ng)
            R.reassemble_groups(pk, seg.stride, ln, plan.total_packets, starts, ng)
        else:
            R.reassemble(pk, seg.stride, ln, plan.total_packets)
        torch.cuda.synchronize()
    got = {r.eventNum: (R.event_bytes(r), r.numFragments) for r in R.poll()}
    st = R.stats()
    return evs, got, {k: int(getattr(st, k)) for k in STATS}, int(st.errorFlags), ngs


CASES = [
    ("mtu1500_205x1mib", [1 << 20] * 205, 1500, 2, False),
    ("mtu1500_ragged", [1, 15, 16, 17, 1435, 1436, 1437, 50000, 3 * 1436, 123457, 0, 1 << 20], 1500, 2, False),
    ("mtu1500_misaligned_v3", [99991, 5, 77777, 1 << 16, (1 << 20) + 3], 1500, 3, True),
    ("mtu9000_1mib", [1 << 20] * 64, 9000, 2, False),
    ("mtu9000_8mib", [8 << 20, 3 << 20, 8936 * 3 + 1], 9000, 2, False),
    ("mtu80_small", [1, 43, 44, 45, 1000, 4321], 80, 2, False),
]


@pytest.mark.parametrize("name,sizes,mtu,ver,mis", CASES, ids=[c[0] for c in CASES])
def test_groups_match_uniform_path(hip, name, sizes, mtu, ver, mis):
    evs, got, st, ef, ngs = _run(hip, sizes, mtu, ver, True, misalign=mis, seed=len(name))
    _, ref, rst, ref_ef, _ = _run(hip, sizes, mtu, ver, False, misalign=mis, seed=len(name))
    assert ef == 0 and ref_ef == 0
    assert st == rst
    # a 0-byte event has no datagrams (numBuffers = 0, e2sarDPSegmenter.cpp:670), so never arrives
    assert set(got) == set(ref) and len(got) == 2 * sum(1 for s in sizes if s > 0)
    for evn, (b, nf) in got.items():
        k = evn % 1000
        assert b == evs[k].tobytes(), f"event {evn} bytes differ"
        assert nf == ref[evn][1]
    if mtu in (1500, 9000) and max(sizes) >= 1 << 16:
        assert all(ng > 0 for ng in ngs), "expected XCD stripes for this batch"


def test_small_mtu_has_no_stripes_and_falls_back(hip):
    """MTU 80 (64-B slots, 128 datagrams per 8-KiB seg unit): a stripe would exceed 64
    datagrams, nGroups = 0 and the uniform groups are used."""
    evs, got, st, ef, ngs = _run(hip, [5000, 31, 1], 80, 2, True, seed=3, launches=1)
    assert ngs == [0]
    assert ef == 0 and st["eventSuccess"] == 3
    for evn, (b, _) in got.items():
        assert b == evs[evn % 1000].tobytes()
