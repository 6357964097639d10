"""The chained form (e2sar_hip_segment_reassemble_batch: segmentation and reassembly of a
batch in one launch, reassembly groups waiting on per-group ready counters) against the
oracle and against the two-launch path.

Bar: the datagrams (bytes and lengths) equal the oracle's segmentation, every event
completes with the source bytes, the counters equal the two-launch path's, and no error
flag is set (bit 4: a group's wait timed out, bit 5: its counter over-counted) -- over
ragged batches, odd and misaligned events, several MTUs and group sizes, LB v2 and v3, and
back-to-back launches (each launch leaves the counters zeroed for the next).
"""
import numpy as np
import pytest

import oracle_ffi as O

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


def _layout(sizes, misalign):
    offs, cur = [], 0
    for k, s in enumerate(sizes):
        cur = (cur + 255) // 256 * 256 + (k % 4 if misalign else 0)
        offs.append(cur)
        cur += s
    return offs, max(cur, 1)


def _run(ctx, sizes, mtu, ver, chained, launches=1, misalign=False, seed=0):
    import torch
    from e2sar_amd import sar
    evs = [_rng_bytes(seed * 1000 + k, s) for k, s in enumerate(sizes)]
    offs, total = _layout(sizes, misalign)
    host = np.zeros(total, np.uint8)
    for e, o in zip(evs, offs):
        host[o:o + len(e)] = e
    dsrc = torch.from_numpy(host).to(ctx.torch_device)
    seg = sar.DeviceSegmenter(ctx, mtu=mtu, lb_hdr_version=ver)
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=1024, queue_capacity=1024,
                              arena_bytes=max(64 << 20, 2 * sum(sizes) + 256 * len(sizes)))
    out = []
    for L in range(launches):
        plan = seg.plan([(dsrc.data_ptr() + o, len(e), 100 * L + k, 7, k, (1 << 40) + k)
                         for k, (e, o) in enumerate(zip(evs, offs))])
        pk, ln = seg.alloc_packets(plan.total_packets)
        if chained:
            seg.segment_reassemble(plan, pk, ln, R)
        else:
            seg.segment(plan, pk, ln)
            R.reassemble(pk, seg.stride, ln, plan.total_packets)
        torch.cuda.synchronize()
        n = plan.total_packets
        got = {r.eventNum: R.event_bytes(r) for r in R.poll()}
        st = R.stats()
        out.append((pk[: n * seg.stride].view(n, seg.stride).cpu().numpy(), ln[:n].cpu().numpy().astype(np.uint32),
                    got, {k: int(getattr(st, k)) for k in STATS}, int(st.errorFlags)))
        R.recycle(force=True)
        R.reset_stats()
    return evs, seg.stride, out


CASES = [
    ("mtu1500_1mib", [1 << 20] * 6, 1500, 2, False),
    ("mtu1500_ragged", [1, 15, 16, 17, 1435, 1436, 1437, 50000, 3 * 1436, 123457, 0], 1500, 2, False),
    ("mtu1500_misaligned_v3", [99991, 5, 77777, 1 << 16], 1500, 3, True),
    ("mtu9000_8mib", [8 << 20, 3 << 20, 8936 * 3 + 1], 9000, 2, False),
    ("mtu80_small", [1, 43, 44, 45, 1000, 4321], 80, 2, False),
    ("mtu104_odd", [777, 12345, 6], 104, 3, True),
]


@pytest.mark.parametrize("name,sizes,mtu,ver,mis", CASES, ids=[c[0] for c in CASES])
def test_chained_matches_oracle_and_two_launches(hip, name, sizes, mtu, ver, mis):
    evs, stride, chained = _run(hip, sizes, mtu, ver, True, launches=2, misalign=mis, seed=len(name))
    _, _, split = _run(hip, sizes, mtu, ver, False, launches=1, misalign=mis, seed=len(name))
    mp = O.max_pld_len(mtu)
    for L, (pk, ln, got, st, flags) in enumerate(chained):
        assert flags == 0, (name, L, flags)
        # datagrams: the oracle's segmentation of the same events
        for k, e in enumerate(evs):
            if len(e) == 0:
                continue
            opk, oln = O.segment_event(e, 100 * L + k, 7, k, (1 << 40) + k, ver, mp, stride)
            base = sum(-(-len(x) // mp) for x in evs[:k])
            m = len(oln)
            assert np.array_equal(ln[base:base + m], oln), (name, L, k)
            for i in range(m):
                assert pk[base + i, :oln[i]].tobytes() == opk[i, :oln[i]].tobytes(), (name, L, k, i)
        # events: every non-empty event back with its bytes
        want = {100 * L + k: e.tobytes() for k, e in enumerate(evs) if len(e)}
        assert got == want, (name, L)
    # counters equal the two-launch path's
    assert chained[0][3] == split[0][3], (name, chained[0][3], split[0][3])
    assert chained[1][3] == split[0][3], name


def test_chained_full_batch_round_trip(hip):
    # the bench's batch: 205 x 1 MiB at MTU 1500 (149,855 datagrams), three launches
    evs, stride, out = _run(hip, [1 << 20] * 205, 1500, 2, True, launches=3, seed=5)
    for L, (pk, ln, got, st, flags) in enumerate(out):
        assert flags == 0 and st["eventSuccess"] == 205 and st["inProgress"] == 0, (L, st, flags)
        assert st["totalPackets"] == 205 * 731
        assert all(got[100 * L + k] == e.tobytes() for k, e in enumerate(evs)), L


@pytest.mark.parametrize("mtu,sizes_per_batch", [
    (1500, [[1 << 20] * 4, [1, 1437, 99991], [5 << 20, 17], [0, 3], [70000] * 9]),
    (80, [[4321, 1], [999] * 3, [45, 44, 43]]),
])
def test_chained_several_batches_one_launch(hip, mtu, sizes_per_batch):
    import torch
    from e2sar_amd import sar
    seg = sar.DeviceSegmenter(hip, mtu=mtu, lb_hdr_version=2)
    R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=1024, queue_capacity=1024, arena_bytes=64 << 20)
    plans, bufs, want, keep = [], [], {}, []
    for b, sizes in enumerate(sizes_per_batch):
        evs = [_rng_bytes(77 * b + k, s) for k, s in enumerate(sizes)]
        offs, total = _layout(sizes, b % 2 == 1)
        host = np.zeros(total, np.uint8)
        for e, o in zip(evs, offs):
            host[o:o + len(e)] = e
        d = torch.from_numpy(host).to(hip.torch_device)
        keep.append(d)
        plans.append(seg.plan([(d.data_ptr() + o, len(e), 1000 * b + k, 3, k, k)
                               for k, (e, o) in enumerate(zip(evs, offs))]))
        bufs.append(seg.alloc_packets(plans[-1].total_packets))
        want.update({1000 * b + k: e.tobytes() for k, e in enumerate(evs) if len(e)})
    for rep in range(2):                        # the second launch reuses the zeroed counters
        seg.segment_reassemble_batches(plans, bufs, R)
        torch.cuda.synchronize()
        got = {r.eventNum: R.event_bytes(r) for r in R.poll()}
        st = R.stats()
        assert int(st.errorFlags) == 0 and got == want, rep
        assert int(st.totalPackets) == sum(p.total_packets for p in plans) and int(st.inProgress) == 0
        # the datagrams of every batch are the oracle's
        mp = O.max_pld_len(mtu)
        for b, (p, (pk, ln)) in enumerate(zip(plans, bufs)):
            n = p.total_packets
            hp = pk[: n * seg.stride].view(n, seg.stride).cpu().numpy()
            hl = ln[:n].cpu().numpy().astype(np.uint32)
            base = 0
            for k, s in enumerate(sizes_per_batch[b]):
                if s == 0:
                    continue
                e = np.frombuffer(want[1000 * b + k], np.uint8)
                opk, oln = O.segment_event(e, 1000 * b + k, 3, k, k, 2, mp, seg.stride)
                m = len(oln)
                assert np.array_equal(hl[base:base + m], oln), (b, k)
                assert all(hp[base + i, :oln[i]].tobytes() == opk[i, :oln[i]].tobytes() for i in range(m)), (b, k)
                base += m
        R.recycle(force=True)
        R.reset_stats()
