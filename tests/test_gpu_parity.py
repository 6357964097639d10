"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar: bit-exact datagrams and event bytes, equal counters.  Sizes are ones the oracle
finishes in seconds; full-size batches are checked through round-trip properties.
"""
import os
import random

import numpy as np
import pytest

import oracle_ffi as O

pytestmark = pytest.mark.gpu

SEND_STR = b"THIS IS A VERY LONG EVENT MESSAGE WE WANT TO SEND EVERY 1 SECONDS."  # reas test :36


def _torch():
    import torch
    return torch


def _rng_bytes(seed, n):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


def _dev(arr, ctx):
    torch = _torch()
    return torch.from_numpy(np.ascontiguousarray(arr)).to(ctx.torch_device)


def _segment_gpu(ctx, events, mtu, ver, offsets=None):
    """events: list of (np bytes, eventNum, dataId, entropy, tick); returns (pk[n,stride], lens[n])."""
    torch = _torch()
    from e2sar_amd import sar
    seg = sar.DeviceSegmenter(ctx, mtu=mtu, lb_hdr_version=ver)
    # pack all events in one device arena; offsets let a test misalign an event on purpose
    offs, cur = [], 0
    for k, (b, *_r) in enumerate(events):
        pad = offsets[k] if offsets else 0
        cur = (cur + 255) // 256 * 256 + pad
        offs.append(cur)
        cur += len(b)
    host = np.zeros(max(cur, 1), np.uint8)
    for (b, *_r), o in zip(events, offs):
        host[o:o + len(b)] = b
    darena = _dev(host, ctx)
    base = darena.data_ptr()
    plan = seg.plan([(base + o, len(b), e, d, en, t) for (b, e, d, en, t), o in zip(events, offs)])
    pk, ln = seg.alloc_packets(plan.total_packets)
    seg.segment(plan, pk, ln)
    torch.cuda.synchronize()
    n = plan.total_packets
    return (pk[: n * seg.stride].view(n, seg.stride).cpu().numpy(), ln[:n].cpu().numpy().astype(np.uint32),
            seg)


def _segment_oracle(events, mtu, ver, stride):
    mp = O.max_pld_len(mtu)
    pks, lns = [], []
    for b, e, d, en, t in events:
        p, l = O.segment_event(np.frombuffer(bytes(b), np.uint8), e, d, en, t, ver, mp, stride)
        pks.append(p)
        lns.append(l)
    if not pks:
        return np.zeros((0, stride), np.uint8), np.zeros(0, np.uint32)
    return np.concatenate(pks), np.concatenate(lns)


def _assert_same_datagrams(gp, gl, op, ol):
    assert gp.shape[0] == op.shape[0], (gp.shape, op.shape)
    np.testing.assert_array_equal(gl, ol)
    for k in range(len(ol)):
        L = int(ol[k])
        if not np.array_equal(gp[k, :L], op[k, :L]):
            bad = np.nonzero(gp[k, :L] != op[k, :L])[0]
            raise AssertionError(f"datagram {k} differs at bytes {bad[:16]} (len {L})")


# ----------------------------------------------------------------------------------
# segmentation parity


@pytest.mark.parametrize("mtu,npk", [(80, 5), (104, 2), (1500, 1)])
def test_seg_send_str_counts_and_bytes(hip, mtu, npk):
    # e2sar_reas_test.cpp:195/254 (MTU 80 -> 5 pkts), e2sar_seg_test.cpp:116/174 (MTU 104 -> 2)
    ev = [(np.frombuffer(SEND_STR, np.uint8), 0, 4321, 0xBEEF, 0x0123456789ABCDEF)]
    gp, gl, seg = _segment_gpu(hip, ev, mtu, 2)
    assert gp.shape[0] == npk
    op, ol = _segment_oracle(ev, mtu, 2, seg.stride)
    _assert_same_datagrams(gp, gl, op, ol)


@pytest.mark.parametrize("mtu,ver,nbytes", [
    (1500, 2, 1 << 20), (1500, 3, 1 << 20), (9000, 2, 1 << 20), (9000, 3, 8 << 20),
    (1500, 2, 100000), (9000, 3, 3 * 8936 + 1), (1500, 3, 1436), (1500, 2, 1437)])
def test_seg_parity_sizes(hip, mtu, ver, nbytes):
    evs = [(_rng_bytes(7 + k, nbytes), k, 4321, 1 + (k * 0x9E37) % 65535, (1 << 48) + k) for k in range(3)]
    gp, gl, seg = _segment_gpu(hip, evs, mtu, ver)
    op, ol = _segment_oracle(evs, mtu, ver, seg.stride)
    _assert_same_datagrams(gp, gl, op, ol)


def test_seg_known_answer_headers(hip):
    # A, v2, eventNum 0, dataId 4321, entropy 0xBEEF, tick 0x0123456789ABCDEF
    ev = [(_rng_bytes(1, 1 << 20), 0, 4321, 0xBEEF, 0x0123456789ABCDEF)]
    gp, gl, _ = _segment_gpu(hip, ev, 1500, 2)
    assert gp.shape[0] == 731
    assert gp[0, :36].tobytes().hex() == "4c4202010000beef0123456789abcdef100010e100000000001000000000000000000000"
    assert gp[1, 16:28].tobytes().hex() == "100010e10000059c00100000"
    assert gp[730, 16:28].tobytes().hex() == "100010e1000ffed800100000"
    assert int(gl[730]) == 36 + 296
    ev = [(_rng_bytes(2, 8 << 20), 7, 4321, 0xBEEF, 0x0123456789ABCDEF)]
    gp, gl, _ = _segment_gpu(hip, ev, 9000, 3)
    assert gp.shape[0] == 939
    assert gp[0, :36].tobytes().hex() == "4c420301cdefbeef0123456789abcdef100010e100000000008000000000000000000007"
    assert int(gl[938]) == 36 + 6640


def test_seg_ragged_batch(hip):
    sizes = [0, 1, 2, 3, 4, 5, 11, 12, 13, 15, 16, 17, 1435, 1436, 1437, 2872, 2873, 65536 + 3, 1 << 20]
    evs = [(_rng_bytes(100 + k, s), 1000 + k, 7 + k, (k * 77) & 0xFFFF, k * 0x100000001) for k, s in enumerate(sizes)]
    for ver in (2, 3):
        gp, gl, seg = _segment_gpu(hip, evs, 1500, ver)
        op, ol = _segment_oracle(evs, 1500, ver, seg.stride)
        _assert_same_datagrams(gp, gl, op, ol)


def test_seg_generic_paths(hip):
    # misaligned event bases and a maxPldLen that is not a multiple of 4 take the byte path
    sizes = [1, 5, 1437, 4099, 100003]
    evs = [(_rng_bytes(300 + k, s), k, 1, 2, 3) for k, s in enumerate(sizes)]
    gp, gl, seg = _segment_gpu(hip, evs, 1500, 2, offsets=[1, 2, 3, 1, 2])
    op, ol = _segment_oracle(evs, 1500, 2, seg.stride)
    _assert_same_datagrams(gp, gl, op, ol)
    gp, gl, seg = _segment_gpu(hip, evs, 1499, 3)                 # maxPld 1435
    op, ol = _segment_oracle(evs, 1499, 3, seg.stride)
    _assert_same_datagrams(gp, gl, op, ol)
    gp, gl, seg = _segment_gpu(hip, evs, 67, 2)                   # maxPld 3
    op, ol = _segment_oracle(evs[:3], 67, 2, seg.stride)
    n3 = op.shape[0]
    _assert_same_datagrams(gp[:n3], gl[:n3], op, ol)


# ----------------------------------------------------------------------------------
# reassembly parity


def _reas_gpu(ctx, pk, ln, with_lb, batches=1, now=0, arena=1 << 28, table=4096, mode="fused", group_size=0):
    """Reassemble datagram rows pk[n, stride] (lens ln) on the GPU; returns ({(ev,d): bytes}, stats, reas).

    mode "fused": one reassemble_batch per batch; "split": classify every batch (in
    arrival order, one work buffer each) before any scatter -- the most decoupled order
    the split API allows."""
    from e2sar_amd import sar
    torch = _torch()
    n, stride = pk.shape
    st16 = (stride + 15) // 16 * 16
    buf = np.zeros((max(n, 1), st16), np.uint8)
    buf[:n, :stride] = pk
    dpk = _dev(buf.reshape(-1), ctx)
    dln = _dev(np.ascontiguousarray(ln, np.uint32).view(np.int32), ctx)
    R = sar.DeviceReassembler(ctx, with_lb_header=with_lb, table_slots=table, arena_bytes=arena,
                              group_size=group_size)
    cuts = np.linspace(0, n, batches + 1).astype(int)
    spans = [(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    if mode == "fused":
        for a, b in spans:
            R.reassemble(dpk[a * st16:], st16, dln[a:], b - a, now_ms=now)
    elif mode == "split":
        works = [R.alloc_work(b - a) for a, b in spans]
        for (a, b), w in zip(spans, works):
            R.classify(dpk[a * st16:], st16, dln[a:], b - a, w, now_ms=now)
        for (a, b), w in zip(spans, works):
            R.scatter(dpk[a * st16:], st16, b - a, w)
    else:
        _pipelined(R, dpk, dln, st16, spans, now)
    torch.cuda.synchronize()
    got = {}
    for rec in R.poll():
        key = (rec.eventNum, rec.dataId)
        assert key not in got
        got[key] = (R.event_bytes(rec), rec.numFragments)
    return got, R.stats(), R


@pytest.fixture(params=["fused", "split", "pipelined"])
def reas_mode(request):
    return request.param


def _pipelined(R, dpk, dln, stride, spans, now=0):
    """classify(0), scatter_classify(0, 1), ..., scatter(last): two work buffers."""
    works = [R.alloc_work(max(b - a for a, b in spans)) for _ in range(2)]
    a0, b0 = spans[0]
    R.classify(dpk[a0 * stride:], stride, dln[a0:], b0 - a0, works[0], now_ms=now)
    for k in range(len(spans)):
        a, b = spans[k]
        if k + 1 < len(spans):
            c, d = spans[k + 1]
            R.scatter_classify(stride, dpk[a * stride:], b - a, works[k % 2],
                               dpk[c * stride:], dln[c:], d - c, works[(k + 1) % 2], now_ms=now)
        else:
            R.scatter(dpk[a * stride:], stride, b - a, works[k % 2])


def _reas_oracle(pk, ln, with_lb, qcap=100000):
    r = O.Reassembler(with_lb, qcap)
    r.push_batch(pk, ln)
    out = {}
    for b, e, d in r.pop_all():
        out[(e, d)] = b
    return out, r.stats(), r


def _events_stream(n_ev, size, mtu, ver=2, seed=0, data_id=4321):
    mp = O.max_pld_len(mtu)
    stride = (36 + mp + 15) // 16 * 16
    evs, pks, lns = [], [], []
    for k in range(n_ev):
        b = _rng_bytes(seed + k, size if np.isscalar(size) else size[k])
        evs.append(b)
        p, l = O.segment_event(b, k, data_id, 1 + k, (1 << 48) + k, ver, mp, stride)
        pks.append(p)
        lns.append(l)
    return evs, np.concatenate(pks), np.concatenate(lns)


def _check_reas(got, st, ref, rst):
    assert set(got) == set(ref), (sorted(got)[:5], sorted(ref)[:5])
    for k in ref:
        assert got[k][0] == ref[k], f"event {k} bytes differ"
    for f in ("eventSuccess", "totalPackets", "totalBytes", "badHeaderDiscards", "dataErrCnt",
              "enqueueLoss", "reassemblyLoss"):
        assert getattr(st, f) == rst[f], (f, getattr(st, f), rst[f])
    assert st.inProgress == rst["inProgress"]


@pytest.mark.parametrize("mtu,size,n_ev", [(1500, 1 << 20, 8), (9000, 1 << 20, 8), (80, 67, 5),
                                           (1500, [1, 1436, 1437, 5000, 100000, 3], 6)])
def test_reas_in_order_with_lb(hip, mtu, size, n_ev, reas_mode):
    evs, pk, ln = _events_stream(n_ev, size, mtu)
    ref, rst, _ = _reas_oracle(pk, ln, True)
    got, st, _ = _reas_gpu(hip, pk, ln, True, mode=reas_mode)
    _check_reas(got, st, ref, rst)
    for k, b in enumerate(evs):
        assert ref[(k, 4321)] == b.tobytes()


def test_reas_without_lb_header(hip, reas_mode):
    evs, pk, ln = _events_stream(4, 50000, 1500)
    pk2 = np.zeros_like(pk)
    pk2[:, : pk.shape[1] - 16] = pk[:, 16:]
    ln2 = ln - 16
    ref, rst, _ = _reas_oracle(pk2, ln2, False)
    got, st, _ = _reas_gpu(hip, pk2, ln2, False, mode=reas_mode)
    _check_reas(got, st, ref, rst)


def test_reas_interleaved_offset0_first(hip, reas_mode):
    # events interleaved and each event's tail fragments shuffled, offset-0 fragment first
    evs, pk, ln = _events_stream(6, 30000, 1500, seed=11)
    order = []
    per = []
    idx = 0
    for k in range(6):
        n = O.num_packets(30000, O.max_pld_len(1500))
        per.append(list(range(idx, idx + n)))
        idx += n
    rnd = random.Random(5)
    firsts = [p[0] for p in per]
    rest = [i for p in per for i in p[1:]]
    rnd.shuffle(rest)
    order = firsts + rest
    pk, ln = pk[order], ln[order]
    ref, rst, _ = _reas_oracle(pk, ln, True)
    for batches in (1, 3, 7):
        got, st, _ = _reas_gpu(hip, pk, ln, True, batches=batches, mode=reas_mode)
        _check_reas(got, st, ref, rst)


def test_reas_bad_and_short_datagrams(hip, reas_mode):
    evs, pk, ln = _events_stream(5, 20000, 1500, seed=21)
    pk = pk.copy()
    ln = ln.copy()
    pk[3, 16] = 0x20          # RE version 2 -> invalid
    pk[9, 17] = 1             # reserved byte set -> invalid
    ln[12] = 30               # shorter than LB+RE headers
    ref, rst, _ = _reas_oracle(pk, ln, True)
    got, st, R = _reas_gpu(hip, pk, ln, True, now=100, mode=reas_mode)
    _check_reas(got, st, ref, rst)
    assert st.badHeaderDiscards == 3
    # incomplete events are reported lost by GC, with their fragment counts
    ro = O.Reassembler(True)
    ro.set_time(100)
    ro.push_batch(pk, ln)
    ro.pop_all()
    ro.set_time(1000)
    ro.gc(500)
    ref_lost = sorted(ro.lost_pop_all())
    R.gc(now_ms=1000, timeout_ms=500)
    lost = sorted((r.eventNum, r.dataId, r.numFragments) for r in R.lost_poll())
    assert lost == ref_lost
    s2 = R.stats()
    assert s2.reassemblyLoss == ro.stats()["reassemblyLoss"] and s2.inProgress == 0


def test_reas_bounds_violation_counted(hip, reas_mode):
    evs, pk, ln = _events_stream(2, 5000, 1500, seed=31)
    pk = pk.copy()
    # rewrite fragment 1's bufferOffset so it overruns the event (reference would overflow)
    pk[1, 20:24] = np.frombuffer((4990).to_bytes(4, "big"), np.uint8)
    ref, rst, _ = _reas_oracle(pk, ln, True)
    got, st, _ = _reas_gpu(hip, pk, ln, True, mode=reas_mode)
    _check_reas(got, st, ref, rst)
    assert st.dataErrCnt == 1


def test_reas_multiple_data_ids_same_event_numbers(hip, reas_mode):
    e1, p1, l1 = _events_stream(4, 9000, 1500, seed=41, data_id=1)
    e2, p2, l2 = _events_stream(4, 9000, 1500, seed=51, data_id=2)
    pk = np.concatenate([p1, p2])
    ln = np.concatenate([l1, l2])
    ref, rst, _ = _reas_oracle(pk, ln, True)
    got, st, _ = _reas_gpu(hip, pk, ln, True, table=64, mode=reas_mode)
    _check_reas(got, st, ref, rst)
    assert len(got) == 8


def test_reas_small_table_collisions(hip, reas_mode):
    # 48 events in flight in a 64-slot table: long probe chains, slots claimed by one key
    # while lanes of the same wave with other keys probe past them, the same key in several
    # runs of one wave (shuffled tails), and events created and completed across batches
    evs, pk, ln = _events_stream(48, 3000, 80, seed=91)       # maxPld 16: 188 datagrams each
    per = O.num_packets(3000, O.max_pld_len(80))
    firsts = [k * per for k in range(48)]
    rest = [i for i in range(len(ln)) if i % per]
    random.Random(9).shuffle(rest)
    order = firsts + rest
    pk, ln = pk[order], ln[order]
    ref, rst, _ = _reas_oracle(pk, ln, True)
    for batches in (1, 5):
        got, st, _ = _reas_gpu(hip, pk, ln, True, batches=batches, table=64, mode=reas_mode)
        _check_reas(got, st, ref, rst)
        assert len(got) == 48 and st.errorFlags == 0


@pytest.mark.parametrize("mtu,group", [(1500, g) for g in (1, 7, 33, 49, 59, 63, 64)] +
                         [(9000, g) for g in (1, 3, 16, 64)])
def test_reas_group_sizes(hip, mtu, group):
    # datagrams per reassembly workgroup other than the power of two the chunk budget gives
    # (the launcher's wave balancing picks e.g. 59 at the bench's 205-event batches): groups
    # that cut through runs, events and the float chunk split, against the oracle -- with the
    # 768-thread kernel (slots of <= 4 KiB) and the 512-thread one (jumbo slots), from part
    # of one copy round to many
    sizes = [70000, 1, 1437, 33333, 100000, 5000, 2873]
    if mtu == 9000:
        sizes = [s * 4 for s in sizes]
    evs, pk, ln = _events_stream(7, sizes, mtu, seed=101)
    starts = np.cumsum([0] + [O.num_packets(s, O.max_pld_len(mtu)) for s in sizes])[:-1].tolist()
    rest = [i for i in range(len(ln)) if i not in starts]
    random.Random(group).shuffle(rest)
    order = starts + rest              # offset 0 first, the rest shuffled
    pk, ln = pk[order], ln[order]
    ref, rst, _ = _reas_oracle(pk, ln, True)
    got, st, _ = _reas_gpu(hip, pk, ln, True, batches=2, mode="fused", group_size=group)
    _check_reas(got, st, ref, rst)
    assert len(got) == 7 and st.errorFlags == 0


def test_reas_queue_and_arena_limits(hip, reas_mode):
    # arena too small for all events: the overflow is an enqueue loss, never a fault
    evs, pk, ln = _events_stream(6, 100000, 1500, seed=61)
    got, st, R = _reas_gpu(hip, pk, ln, True, arena=3 * 100096, mode=reas_mode)
    assert st.eventSuccess == 6
    assert len(got) == 3 and st.enqueueLoss == 3
    assert st.errorFlags & 2
    for (e, d), (b, nf) in got.items():
        assert b == evs[e].tobytes()


# ----------------------------------------------------------------------------------
# full-size round trips (size-independent properties)


@pytest.mark.parametrize("mtu,size,n_ev,ver", [(1500, 1 << 20, 96, 2), (9000, 8 << 20, 12, 3)])
def test_roundtrip_full_size(hip, mtu, size, n_ev, ver, reas_mode):
    torch = _torch()
    from e2sar_amd import sar
    g = torch.Generator(device=hip.torch_device)
    g.manual_seed(1234)
    src = torch.randint(0, 256, (n_ev, size), dtype=torch.uint8, device=hip.torch_device, generator=g)
    seg = sar.DeviceSegmenter(hip, mtu=mtu, lb_hdr_version=ver)
    plan = seg.plan([(src[k].data_ptr(), size, k, 4321, 1 + k, (1 << 48) + k) for k in range(n_ev)])
    pk, ln = seg.alloc_packets(plan.total_packets)
    seg.segment(plan, pk, ln)
    R = sar.DeviceReassembler(hip, with_lb_header=True, arena_bytes=n_ev * ((size + 255) // 256 * 256) + 4096)
    work = R.alloc_work(plan.total_packets)

    def reassemble():
        n = plan.total_packets
        if reas_mode == "fused":
            R.reassemble(pk, seg.stride, ln, n)
        elif reas_mode == "split":
            R.classify(pk, seg.stride, ln, n, work)
            R.scatter(pk, seg.stride, n, work)
        else:
            # four batches that cut through events, scatter of k beside classify of k+1
            cuts = [0, n // 4 + 3, n // 2 + 11, 3 * n // 4 + 5, n]
            _pipelined(R, pk, ln, seg.stride, list(zip(cuts[:-1], cuts[1:])))

    reassemble()
    recs = R.poll()
    st = R.stats()
    assert st.eventSuccess == n_ev and len(recs) == n_ev and st.inProgress == 0
    assert st.totalPackets == plan.total_packets == n_ev * O.num_packets(size, seg.max_pld)
    arena = R.arena_tensor()
    for rec in recs:
        assert rec.numFragments == O.num_packets(size, seg.max_pld)
        out = arena[rec.arenaOffset: rec.arenaOffset + rec.bytes]
        assert torch.equal(out, src[rec.eventNum]), f"event {rec.eventNum} differs"
    # recycle and go again: same results from a clean table
    R.recycle(force=False)
    reassemble()
    assert len(R.poll()) == n_ev


def test_reas_compaction_keeps_partial_events(hip):
    # streaming: events straddle two batches; completed records are polled, the arena is
    # compacted, and the partial events finish in the new arena with the right bytes
    torch = _torch()
    from e2sar_amd import sar
    evs, pk, ln = _events_stream(6, 50000, 1500, seed=71)
    n, stride = pk.shape
    st16 = (stride + 15) // 16 * 16
    buf = np.zeros((n, st16), np.uint8)
    buf[:, :stride] = pk
    dpk = _dev(buf.reshape(-1), hip)
    dln = _dev(np.ascontiguousarray(ln, np.uint32).view(np.int32), hip)
    R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=64, arena_bytes=1 << 20, compactable=True)
    cut = n // 2 + 7                      # inside event 3
    R.reassemble(dpk, st16, dln, cut)
    first = {r.eventNum: R.event_bytes(r) for r in R.poll()}
    before = R.stats()
    # the occupancy counters are sharded on the device (ReasOcc); stats() sums them
    assert before.inProgress == 1 and before.tableUsed == 4
    R.compact()
    assert R.stats().tableUsed == 1 and R.stats().inProgress == 1   # only the live event moved
    R.reassemble(dpk[cut * st16:], st16, dln[cut:], n - cut)
    second = {r.eventNum: R.event_bytes(r) for r in R.poll()}
    got = {**first, **second}
    assert sorted(got) == list(range(6))
    for k, b in enumerate(evs):
        assert got[k] == b.tobytes()
    st = R.stats()
    assert st.eventSuccess == 6 and st.inProgress == 0 and st.arenaUsed < before.arenaUsed + 3 * 50176
    assert st.tableUsed == 3
    R.recycle(force=False)
    st = R.stats()
    assert st.tableUsed == 0 and st.inProgress == 0 and st.eventSuccess == 6


@pytest.mark.parametrize("mode", ["fused", "split", "pipelined", "reference_order"])
def test_reas_owner_filter_takes_only_owned_events(hip, mode):
    # e2sar_hip_reas_set_owner: a reassembler of rank r in a world of 3 reassembles exactly
    # the events with eventNum % 3 == r and counts nothing of the others; unparsable
    # datagrams are still counted where they are seen.  Oracle: the same batch restricted
    # to the datagrams the rank keeps.
    from e2sar_amd import _capi
    world = 3
    sizes = [70000, 1, 1437, 33333, 100000, 5000, 2873, 9000, 12345, 1436, 64000]
    evs, pk, ln = _events_stream(len(sizes), sizes, 1500, seed=131)
    starts = np.cumsum([0] + [O.num_packets(s, O.max_pld_len(1500)) for s in sizes])[:-1].tolist()
    rest = [i for i in range(len(ln)) if i not in starts]
    random.Random(17).shuffle(rest)
    order = starts + rest
    pk, ln = pk[order].copy(), ln[order].copy()
    bad_ev = int.from_bytes(pk[len(ln) // 2, 28:36].tobytes(), "big")
    pk[len(ln) // 2, 16] = 0x20                      # one unparsable datagram: its event never completes
    keys = [O.re_parse(pk[k, 16:36].tobytes()) for k in range(len(ln))]
    for r in range(world):
        keep = np.array([not ok or e % world == r for ok, _, _, _, e, _ in keys], bool)
        ref, rst, _ = _reas_oracle(pk[keep], ln[keep], True)
        if mode == "reference_order":
            from e2sar_amd import sar
            torch = _torch()
            n, stride = pk.shape
            dpk = _dev(pk.reshape(-1), hip)
            dln = _dev(np.ascontiguousarray(ln, np.uint32).view(np.int32), hip)
            R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=256, arena_bytes=1 << 24,
                                      flags=_capi.REAS_REFERENCE_ORDER)
            R.set_owner(world, r)
            R.reassemble(dpk, stride, dln, n)
            torch.cuda.synchronize()
            got = {(x.eventNum, x.dataId): (R.event_bytes(x), x.numFragments) for x in R.poll()}
            st = R.stats()
        else:
            got, st, R = _owner_reas(hip, pk, ln, world, r, mode)
        _check_reas(got, st, ref, rst)
        assert sorted(e for e, _ in got) == [k for k in range(len(sizes)) if k % world == r and k != bad_ev]
        assert st.badHeaderDiscards == 1 and st.errorFlags == 0


def _owner_reas(ctx, pk, ln, world, rank, mode):
    from e2sar_amd import sar
    torch = _torch()
    n, stride = pk.shape
    dpk = _dev(pk.reshape(-1), ctx)
    dln = _dev(np.ascontiguousarray(ln, np.uint32).view(np.int32), ctx)
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=256, arena_bytes=1 << 24)
    R.set_owner(world, rank)
    cuts = [0, n // 3 + 1, 2 * n // 3 + 5, n]
    spans = list(zip(cuts[:-1], cuts[1:]))
    if mode == "fused":
        for a, b in spans:
            R.reassemble(dpk[a * stride:], stride, dln[a:], b - a)
    elif mode == "split":
        R.set_cold(True)
        for a, b in spans:
            w = R.alloc_work(b - a)
            R.classify(dpk[a * stride:], stride, dln[a:], b - a, w)
            R.scatter(dpk[a * stride:], stride, b - a, w)
    else:
        _pipelined(R, dpk, dln, stride, spans)
    torch.cuda.synchronize()
    got = {(x.eventNum, x.dataId): (R.event_bytes(x), x.numFragments) for x in R.poll()}
    return got, R.stats(), R


@pytest.mark.parametrize("world,self_rank", [(3, 0), (8, 5)])
def test_route_foreign_skips_owned(hip, world, self_rank):
    # foreign-only routing == the stable owner packing with this rank's share (and the
    # unparsable datagram) left out; counts[self] == 0
    from test_dist_gloo import stable_route
    from e2sar_amd.dist import PacketRouter
    evs, pk, ln = _events_stream(20, 7000, 1500, seed=83)
    perm = np.random.default_rng(6).permutation(len(ln))
    pk, ln = pk[perm].copy(), ln[perm].copy()
    pk[3, 16] = 0x20
    n, stride = pk.shape
    dpk = _dev(pk.reshape(-1), hip)
    dln = _dev(np.ascontiguousarray(ln, np.uint32).view(np.int32), hip)
    router = PacketRouter(hip, stride, n, world, self_rank)
    spk, sln, cnt = router.route(dpk, dln, n, foreign_only=True)
    _torch().cuda.synchronize()
    rpk, rln, rcounts = stable_route(pk, ln, world, self_rank)
    # drop this rank's span from the stable packing
    base = sum(rcounts[:self_rank])
    m = rcounts[self_rank]
    rcounts = list(rcounts)
    rcounts[self_rank] = 0
    rpk = np.concatenate([rpk[:base], rpk[base + m:]])
    rln = np.concatenate([rln[:base], rln[base + m:]])
    assert cnt.cpu().tolist() == rcounts
    k = len(rln)
    np.testing.assert_array_equal(sln[:k].cpu().numpy().astype(np.uint32), rln)
    np.testing.assert_array_equal(spk[: k * stride].cpu().numpy().reshape(k, stride), rpk)


@pytest.mark.parametrize("world,self_rank", [(2, 1), (8, 3)])
def test_route_batch_matches_stable_route(hip, world, self_rank):
    # gfx950 route kernels == the host restatement of the stable owner packing
    from test_dist_gloo import stable_route
    from e2sar_amd.dist import PacketRouter
    evs, pk, ln = _events_stream(20, 7000, 1500, seed=81)
    perm = np.random.default_rng(5).permutation(len(ln))      # arbitrary landing order
    pk, ln = pk[perm].copy(), ln[perm].copy()
    pk[3, 16] = 0x20                                          # one unparsable datagram stays home
    n, stride = pk.shape
    dpk = _dev(pk.reshape(-1), hip)
    dln = _dev(np.ascontiguousarray(ln, np.uint32).view(np.int32), hip)
    router = PacketRouter(hip, stride, n, world, self_rank)
    spk, sln, cnt = router.route(dpk, dln, n)
    _torch().cuda.synchronize()
    rpk, rln, rcounts = stable_route(pk, ln, world, self_rank)
    assert cnt.cpu().tolist() == rcounts
    np.testing.assert_array_equal(sln[:n].cpu().numpy().astype(np.uint32), rln)
    got = spk[: n * stride].cpu().numpy().reshape(n, stride)
    np.testing.assert_array_equal(got, rpk)


def test_relay_resegments_completed_events(hip):
    # BASELINE config 5 on the device: segment -> reassemble -> relay_plan -> segment_device.
    # Every re-sent datagram equals the oracle's segmentation of the reassembled event with
    # the relay's rules (RE eventNum and dataId as received, one LB tick, entropy base + i)
    torch = _torch()
    from e2sar_amd import sar
    sizes = [1, 1436, 1437, 3 * 1436 + 5, 100_000, 1 << 20]
    host = [_rng_bytes(500 + k, s) for k, s in enumerate(sizes)]
    evs = [(b, 10 + k, 7, 1 + k, 99 + k) for k, b in enumerate(host)]
    gp, gl, seg = _segment_gpu(hip, evs, 1500, 2)
    R = sar.DeviceReassembler(hip, with_lb_header=True, arena_bytes=8 << 20)
    dpk = _dev(gp.reshape(-1), hip)
    dln = _dev(gl.view(np.int32), hip)
    R.reassemble(dpk, seg.stride, dln, gp.shape[0])
    n_ev = len(sizes)
    mp = O.max_pld_len(1500)
    max_pk = max(O.num_packets(s, mp) for s in sizes)
    d_events = torch.zeros(n_ev * sar.SEG_EVENT_BYTES, dtype=torch.uint8, device=hip.torch_device)
    counts = torch.zeros(2, dtype=torch.int32, device=hip.torch_device)
    tick = 0x0102030405060708
    R.relay_plan(d_events, counts, 0, n_ev, mp, tick, 0xFFFE)          # entropy wraps past 0xFFFF
    out = sar.DeviceSegmenter(hip, mtu=1500, lb_hdr_version=3)
    opk, oln = out.alloc_packets(n_ev * max_pk)
    out.segment_device(d_events, counts, n_ev, max_pk, opk, oln)
    torch.cuda.synchronize()
    n, total = (int(x) for x in counts.cpu())
    assert n == n_ev and total == sum(O.num_packets(s, mp) for s in sizes)
    dt = np.dtype([("data", "<u8"), ("eventNum", "<u8"), ("lbTick", "<u8"), ("bytes", "<u4"), ("pktBase", "<u4"),
                   ("dataId", "<u2"), ("entropy", "<u2"), ("reserved", "<u4")])
    desc = d_events.cpu().numpy().view(dt)
    got_pk = opk[: total * out.stride].view(total, out.stride).cpu().numpy()
    got_ln = oln[:total].cpu().numpy().astype(np.uint32)
    assert sorted(int(d["eventNum"]) for d in desc) == [10 + k for k in range(n_ev)]
    for i, d in enumerate(desc):
        k = int(d["eventNum"]) - 10
        assert int(d["bytes"]) == sizes[k] and int(d["dataId"]) == 7 and int(d["lbTick"]) == tick
        assert int(d["entropy"]) == (0xFFFE + i) & 0xFFFF
        op, ol = O.segment_event(host[k], 10 + k, 7, (0xFFFE + i) & 0xFFFF, tick, 3, mp, out.stride)
        b = int(d["pktBase"])
        _assert_same_datagrams(got_pk[b:b + len(ol)], got_ln[b:b + len(ol)], op, ol)


# ----------------------------------------------------------------------------------
# seeded random workloads, end to end


@pytest.mark.parametrize("seed", range(int(os.environ.get("E2SAR_RANDOM_SEEDS", "8"))))
def test_random_workload_segment_then_reassemble(hip, seed):
    # random event sizes (edge sizes included), MTU, LB version, dataIds, 40-bit event
    # numbers, 64-bit ticks and misaligned event buffers; the GPU's datagrams must equal the
    # oracle's, then those datagrams -- all events interleaved, offset 0 first per event
    # (DESIGN.md 5.3), cut into random batches -- reassemble to the oracle's events and
    # counters in a random launch form
    rnd = random.Random(1000 + seed)
    mtu = rnd.choice([80, 104, 576, 1499, 1500, 4000, 9000])
    ver = rnd.choice([2, 3])
    cap = 150_000 if mtu >= 1499 else 20_000
    # every fourth seed at MTU >= 1499 draws events up to 8 MiB, so the fused kernel's
    # deferred run-tail add (events >= E2SAR_REAS_DEFER_ACC = 4 MiB) meets random workloads
    big = seed % 4 == 3 and mtu >= 1499
    if big:
        cap = 8 << 20
    evs, keys = [], set()
    while len(evs) < (rnd.randint(1, 4) if big else rnd.randint(1, 12)):
        size = rnd.choice([1, 3, 4, 17, 1435, 1436, 1437]) if rnd.random() < 0.3 else rnd.randint(1, cap)
        if big and len(evs) == 0:
            size = rnd.randint(4 << 20, 8 << 20)
        e, d = rnd.randint(0, (1 << 40) - 1), rnd.choice([1, 2, 4321])
        if (e, d) in keys:
            continue
        keys.add((e, d))
        evs.append((_rng_bytes(seed * 100 + len(evs), size), e, d, rnd.randint(0, 65535), rnd.getrandbits(64)))
    offsets = [rnd.randint(0, 255) for _ in evs]
    gp, gl, seg = _segment_gpu(hip, evs, mtu, ver, offsets=offsets)
    op, ol = _segment_oracle(evs, mtu, ver, seg.stride)
    _assert_same_datagrams(gp, gl, op, ol)

    per = [O.num_packets(len(b), O.max_pld_len(mtu)) for b, *_r in evs]
    starts = np.cumsum([0] + per)[:-1].tolist()
    first = set(starts)
    rest = [i for i in range(len(ol)) if i not in first]
    rnd.shuffle(rest)
    order = starts + rest
    pk, ln = gp[order], gl[order]
    ref, rst, _ = _reas_oracle(pk, ln, True)
    for b, e, d, *_r in evs:
        assert ref[(e, d)] == b.tobytes()
    mode = rnd.choice(["fused", "split", "pipelined"])
    got, st, _ = _reas_gpu(hip, pk, ln, True, batches=rnd.randint(1, 4), mode=mode)
    _check_reas(got, st, ref, rst)
    assert len(got) == len(evs) and st.errorFlags == 0


def _singleton_at(order_len, batches, group, pos):
    """True when datagram `pos` of a stream of order_len, cut into `batches` linspace batches
    of fused groups of `group`, is the last datagram of its group (its run cannot extend
    past it)."""
    cuts = np.linspace(0, order_len, batches + 1).astype(int)
    for a, b in zip(cuts[:-1], cuts[1:]):
        if a <= pos < b:
            return (pos - a + 1) % group == 0 or pos + 1 == b
    return False


@pytest.mark.parametrize("mtu", [1500, 9000])
@pytest.mark.parametrize("batches,group", [(1, 49), (3, 64), (1, 7), (2, 16)])
def test_reas_large_events_with_loss_fused(hip, mtu, batches, group):
    # events of 4-8 MiB through the fused reas_kernel, where run tails of events of at
    # least 4 MiB add to the accumulator after the copy (E2SAR_REAS_DEFER_ACC,
    # sar_kernels.hip reas_range): A loses one datagram to a bad RE version (never
    # completes, GC reports it lost), B receives one full datagram twice, in its middle
    # (curBytes passes its length without meeting it, so it never completes -- the
    # reference's rule, cpp:398-403), C arrives with its tail shuffled, D intact.  Events,
    # bytes, every counter and the lost records equal the oracle's
    # (e2sarDPReassembler.cpp:331-427).
    # The device adds per run, in any order: B could meet its length only if its last add
    # were a run of exactly one full datagram, which needs B's first datagram alone in its
    # group; A's tail is trimmed until the cuts do not isolate it (asserted below).
    sizes = [4 << 20, (6 << 20) + 13, (8 << 20) - 5, 8 << 20]
    evs, pk, ln = _events_stream(4, sizes, mtu, seed=70 + mtu)
    mp = O.max_pld_len(mtu)
    per = [O.num_packets(z, mp) for z in sizes]
    assert (sizes[1] - (per[1] - 1) * mp) != mp               # B's tail is short
    st = np.cumsum([0] + per)
    pk, ln = pk.copy(), ln.copy()
    pk[st[0] + per[0] // 2, 16] = 0x20                           # A: RE version 2 -> invalid
    rnd = random.Random(mtu)
    c_idx = list(range(st[2], st[3]))
    tail = c_idx[1:]
    rnd.shuffle(tail)                                            # C: offset 0 first, tail shuffled
    b_idx = list(range(st[1], st[2]))
    dup = b_idx[len(b_idx) // 3]                                 # B: one full datagram twice
    b_order = b_idx[: len(b_idx) // 2] + [dup] + b_idx[len(b_idx) // 2:]
    a_n = per[0]
    while True:
        order = list(range(st[0], st[0] + a_n)) + b_order + [c_idx[0]] + tail + list(range(st[3], st[4]))
        if not _singleton_at(len(order), batches, group, a_n):
            break
        a_n -= 1
    assert a_n > per[0] // 2 + 1                                 # A keeps its bad datagram
    pk, ln = pk[order], ln[order]
    ref, rst, _ = _reas_oracle(pk, ln, True)
    assert set(ref) == {(2, 4321), (3, 4321)}
    got, stt, R = _reas_gpu(hip, pk, ln, True, batches=batches, now=100, arena=64 << 20,
                            mode="fused", group_size=group)
    _check_reas(got, stt, ref, rst)
    assert stt.badHeaderDiscards == 1 and stt.errorFlags == 0
    assert got[(2, 4321)][0] == evs[2].tobytes() and got[(3, 4321)][0] == evs[3].tobytes()
    ro = O.Reassembler(True)
    ro.set_time(100)
    ro.push_batch(pk, ln)
    ro.pop_all()
    ro.set_time(1000)
    ro.gc(500)
    R.gc(now_ms=1000, timeout_ms=500)
    assert sorted((r.eventNum, r.dataId, r.numFragments) for r in R.lost_poll()) == sorted(ro.lost_pop_all())


def test_duplicate_inside_a_run_default_vs_reference_order(hip):
    """Pins where the default device path departs from the reference under a duplicate
    (DESIGN 5.3).  The reference tests completion after every fragment (cpp:398-403): with
    arrival d0, d2, d3, d4 (tail), d1, d1 it meets the event's length at d1 -- the event
    completes, whole -- and the repeated d1 opens a new item that never completes.  The
    default device path adds per run of equal keys: the six datagrams are one run in one
    group, whose single add (83 bytes) passes the 67-byte length without meeting it, so the
    event stays in progress.  REFERENCE_ORDER mode gives the reference's result exactly."""
    from e2sar_amd import _capi, sar
    torch = _torch()
    evs, pk, ln = _events_stream(1, len(SEND_STR), 80)
    assert pk.shape[0] == 5
    order = [0, 2, 3, 4, 1, 1]
    pk, ln = pk[order], ln[order]
    ref, rst, _ = _reas_oracle(pk, ln, True)
    assert set(ref) == {(0, 4321)} and ref[(0, 4321)] == evs[0].tobytes()
    assert rst["eventSuccess"] == 1 and rst["inProgress"] == 1   # the repeated d1's own item
    got, st, _ = _reas_gpu(hip, pk, ln, True, group_size=64)
    assert got == {} and st.eventSuccess == 0 and st.inProgress == 1
    assert st.totalPackets == 6 and st.badHeaderDiscards == 0 and st.dataErrCnt == 0
    # reference-order mode: the reference's events and counters
    n, stride = pk.shape
    dpk = _dev(pk.reshape(-1), hip)
    dln = _dev(np.ascontiguousarray(ln, np.uint32).view(np.int32), hip)
    R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=64, arena_bytes=1 << 20,
                              flags=_capi.REAS_REFERENCE_ORDER)
    R.reassemble(dpk, stride, dln, n)
    torch.cuda.synchronize()
    recs = R.poll()
    assert [(r.eventNum, r.dataId) for r in recs] == [(0, 4321)]
    assert R.event_bytes(recs[0]) == ref[(0, 4321)]
    _check_reas({(0, 4321): (R.event_bytes(recs[0]), recs[0].numFragments)}, R.stats(), ref, rst)
