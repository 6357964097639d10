"""Reference-order reassembly (E2SAR_HIP_REAS_REFERENCE_ORDER) against the oracle.

With the flag the device applies the reference receive body's arrival-order rules
(e2sarDPReassembler.cpp:361-427): offset 0 always starts a new item and drops the one in
progress, a fragment after completion starts an item of its own, completion is tested
after every fragment.  Bar: for ANY arrival order -- duplicates, late offset-0 fragments,
drops, replays after completion, bad headers -- the completed events, their bytes, every
counter and the GC's lost records equal the oracle's sequential restatement, in every
launch form and batch cut.
"""
import json
import os
import random

import numpy as np
import pytest

import oracle_ffi as O
from test_gpu_golden import GOLDEN, STATS, _expected, _reas_case

pytestmark = pytest.mark.gpu


def _flag():
    from e2sar_amd import _capi
    return _capi.REAS_REFERENCE_ORDER


@pytest.mark.parametrize("mode", ["fused", "split"])
@pytest.mark.parametrize("per_datagram", [True, False])
def test_golden_reassembly_reference_order(hip, mode, per_datagram):
    with open(GOLDEN) as f:
        golden = json.load(f)
    for case in golden["reassemble"]:
        got, st, lost = _reas_case(hip, case, mode, per_datagram, flags=_flag())
        if case.get("deviceRingCapacity") and not per_datagram:
            # which two of three events completed in one launch fit the 2-record ring is the
            # device's completion order; counts and bytes still match
            assert st == case["stats"]
            assert len(got) == 2 and all(got[k] == h for k, h in _expected(case).items() if k in got)
            continue
        assert got == _expected(case), case["name"]
        assert st == case["stats"], (case["name"], st, case["stats"])


def _completes_with_a_hole(pk, ln):
    """True if, taken in arrival order with the reference's rules, some event completes
    while part of its buffer was never written (a duplicate standing in for a fragment that
    was dropped or went to a replaced item): those bytes are whatever the buffer held
    (uninitialised in the reference, cpp:391) and cannot be compared."""
    items = {}
    for p in range(len(ln)):
        if int(ln[p]) < 36:
            continue
        ok, d, off, blen, ev, _ = O.re_parse(pk[p, 16:36].tobytes())
        pl = int(ln[p]) - 36
        if not ok or off + pl > blen:
            continue
        it = items.get((ev, d))
        if off == 0 or it is None:
            it = items[(ev, d)] = [blen, 0, np.zeros(blen, bool)]
        it[1] += pl
        it[2][off:off + pl] = True
        if it[1] == it[0]:
            if not it[2].all():
                return True
            items[(ev, d)] = None
    return False


def _stream(seed):
    """A random arrival stream: events of random sizes fragmented at a random MTU, then
    interleaved with duplicates, late offset-0 fragments, drops, replays and bad headers
    (redrawn until no event would complete with a hole)."""
    for sub in range(1000):
        out = _draw(seed * 1000 + sub)
        if not _completes_with_a_hole(out[0], out[1]):
            return out
    raise AssertionError("no hole-free stream drawn")


def _draw(seed):
    rnd = random.Random(seed)
    mtu = rnd.choice([80, 104, 200, 1500])
    mp = O.max_pld_len(mtu)
    stride = (36 + mp + 15) // 16 * 16
    per_event = []
    for k in range(rnd.randint(3, 14)):
        size = rnd.choice([1, 15, 16, 17, 67, mp, mp + 1]) if rnd.random() < 0.3 else rnd.randint(1, 40 * mp)
        ev = np.random.default_rng(seed * 131 + k).integers(0, 256, size, dtype=np.uint8)
        pk, ln = O.segment_event(ev, (1000 + k) * rnd.choice([1, 1 << 33]), rnd.choice([1, 4321]), 7, 99, 2, mp, stride)
        frags = [(pk[i].copy(), int(ln[i])) for i in range(len(ln))]
        order = list(range(len(frags)))
        r = rnd.random()
        if r < 0.35:
            rnd.shuffle(order)                                  # out of order, offset 0 anywhere
        elif r < 0.5 and len(order) > 1:
            j = rnd.randint(2, len(order))
            order = order[1:j] + [0] + order[j:]                                      # late offset 0
        seq = [frags[i] for i in order]
        r2 = rnd.random()
        if r2 < 0.3 and seq:
            seq.insert(rnd.randint(0, len(seq)), seq[rnd.randrange(len(seq))])        # a duplicate
        elif r2 < 0.45 and len(seq) > 1:
            seq.pop(rnd.randrange(len(seq)))                                          # a drop
        if rnd.random() < 0.15:
            seq += [frags[i] for i in range(rnd.randint(1, len(frags)))]              # replay after completion
        per_event.append(seq)
    # interleave the events' streams, keeping each stream's own order
    out = []
    while any(per_event):
        s = rnd.choice([s for s in per_event if s])
        out.append(s.pop(0))
    for _ in range(rnd.randint(0, 3)):                                                # bad headers
        pk, L = out[rnd.randrange(len(out))]
        bad = pk.copy()
        bad[16] = 0x20
        out.insert(rnd.randint(0, len(out)), (bad, L))
    pk = np.stack([p for p, _ in out])
    ln = np.array([L for _, L in out], np.uint32)
    return pk, ln, stride, rnd


def _gpu(ctx, pk, ln, stride, cuts, mode, now0=100, arena=64 << 20, slots=256):
    import torch
    from e2sar_amd import sar
    n = len(ln)
    dpk = torch.from_numpy(np.ascontiguousarray(pk).reshape(-1)).to(ctx.torch_device)
    dln = torch.from_numpy(ln.view(np.int32).copy()).to(ctx.torch_device)
    R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=slots, queue_capacity=4096, lost_capacity=4096,
                              arena_bytes=arena, flags=_flag())
    spans = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    works = [R.alloc_work(n) for _ in range(2)]
    if mode == "pipelined":
        a0, b0 = spans[0]
        R.classify(dpk[a0 * stride:], stride, dln[a0:], b0 - a0, works[0], now_ms=now0)
        for k, (a, b) in enumerate(spans):
            if k + 1 < len(spans):
                c, d = spans[k + 1]
                R.scatter_classify(stride, dpk[a * stride:], b - a, works[k % 2], dpk[c * stride:], dln[c:], d - c,
                                   works[(k + 1) % 2], now_ms=now0)
            else:
                R.scatter(dpk[a * stride:], stride, b - a, works[k % 2])
    else:
        for k, (a, b) in enumerate(spans):
            if mode == "fused":
                R.reassemble(dpk[a * stride:], stride, dln[a:], b - a, now_ms=now0)
            else:
                R.classify(dpk[a * stride:], stride, dln[a:], b - a, works[k % 2], now_ms=now0)
                R.scatter(dpk[a * stride:], stride, b - a, works[k % 2])
    torch.cuda.synchronize()
    got = {}
    for rec in R.poll():
        got.setdefault((rec.eventNum, rec.dataId), []).append((R.event_bytes(rec), rec.numFragments))
    st = R.stats()
    R.gc(now_ms=now0 + 1000, timeout_ms=500)
    lost = sorted((r.eventNum, r.dataId, r.numFragments) for r in R.lost_poll())
    st2 = R.stats()
    return got, {k: int(getattr(st, k)) for k in STATS}, lost, int(st2.reassemblyLoss), int(st2.inProgress)


def _oracle(pk, ln):
    r = O.Reassembler(True, 1 << 20)
    r.set_time(100)
    r.push_batch(pk, ln)
    got = {}
    for b, e, d, nf in r.pop_all_frags():
        got.setdefault((e, d), []).append((b, nf))
    st = r.stats()
    r.set_time(1100)
    r.gc(500)
    lost = sorted(r.lost_pop_all())
    st2 = r.stats()
    return got, {k: int(st[k]) for k in STATS}, lost, int(st2["reassemblyLoss"]), int(st2["inProgress"])


@pytest.mark.parametrize("seed", range(int(os.environ.get("E2SAR_RANDOM_SEEDS", "12"))))
def test_random_arrival_orders_match_the_reference(hip, seed):
    pk, ln, stride, rnd = _stream(seed)
    ref, rst, rlost, rloss, rinp = _oracle(pk, ln)
    n = len(ln)
    nb = rnd.randint(1, 5)
    cuts = sorted({0, n, *[rnd.randint(0, n) for _ in range(nb - 1)]})
    mode = ["fused", "split", "pipelined"][seed % 3]
    got, st, lost, loss, inp = _gpu(hip, pk, ln, stride, cuts, mode)
    assert st == rst, (mode, st, rst)
    assert sorted(got) == sorted(ref), mode
    for k in ref:
        # bytes AND numFragments of every completed item (the walk counts duplicates, as
        # cpp:398 does; the random streams keep one bufferLength per key, so no fragment
        # overruns its item)
        assert sorted(got[k]) == sorted(ref[k]), (k, mode)
    assert lost == rlost and loss == rloss and inp == rinp == 0


@pytest.mark.parametrize("mode", ["fused", "pipelined"])
def test_large_events_shuffled_with_duplicates(hip, mode):
    # 1 MiB events at MTU 1500, tails shuffled, a few duplicates and one late offset 0: every
    # key files far more than kRoBucket runs per batch (the overflow placement and sort of
    # ro_place_kernel); pipelined: each batch's key pass + walk beside the previous scatter
    rnd = random.Random(77)
    mp = O.max_pld_len(1500)
    stride = (36 + mp + 15) // 16 * 16
    seqs = []
    for k in range(6):
        ev = np.random.default_rng(500 + k).integers(0, 256, 1 << 20, dtype=np.uint8)
        pk, ln = O.segment_event(ev, k, 4321, 1, 2, 2, mp, stride)
        order = list(range(len(ln)))
        rnd.shuffle(order)
        if k == 2:
            order.insert(300, order[5])           # duplicate: never completes
        seqs.append([(pk[i], int(ln[i])) for i in order])
    out = []
    while any(seqs):
        s = rnd.choice([s for s in seqs if s])
        out.append(s.pop(0))
    pk = np.stack([p for p, _ in out])
    ln = np.array([L for _, L in out], np.uint32)
    ref, rst, rlost, rloss, rinp = _oracle(pk, ln)
    n = len(ln)
    got, st, lost, loss, inp = _gpu(hip, pk, ln, stride, [0, n // 3, n // 2, 5 * n // 6, n], mode)
    assert st == rst and sorted(got) == sorted(ref)
    for k in ref:
        assert sorted(got[k]) == sorted(ref[k])              # bytes and numFragments
    assert lost == rlost and loss == rloss


@pytest.mark.parametrize("nev,ev_bytes,slots", [(3, 1 << 20, 256), (2, 5 << 20, 256), (3, 1 << 20, 32768)])
def test_interleaved_events_many_runs(hip, nev, ev_bytes, slots):
    """Events interleaved datagram by datagram (concurrent senders): every run of one key is
    one datagram long, so each key files hundreds to thousands of runs -- its bucket
    overflows, the runs are placed by their index and sorted by the key's walk wave (in LDS
    up to 2048 runs: 3 x 1 MiB, 731 runs each; in global memory above: 2 x 5 MiB, 3651 runs
    each).  A late offset 0 and a duplicate ride along.  slots 32768: a table above
    ro_place_kernel's LDS scan (kPlaceLdsSlots, 16384 slots), whose overflow runs are then
    scanned and placed through the global runBase by workgroup 0."""
    rnd = random.Random(nev)
    mp = O.max_pld_len(1500)
    stride = (36 + mp + 15) // 16 * 16
    seqs = []
    for k in range(nev):
        ev = np.random.default_rng(700 + k).integers(0, 256, ev_bytes, dtype=np.uint8)
        pk, ln = O.segment_event(ev, 90 + k, 4321, 1, 2, 2, mp, stride)
        order = list(range(len(ln)))
        if k == 0:
            order = order[1:40] + [0] + order[40:]            # late offset 0: the first 39 are orphaned
        if k == 1:
            order.insert(500, order[77])                      # a duplicate before the end
        seqs.append([(pk[i], int(ln[i])) for i in order])
    out = []
    while any(seqs):                                          # round robin over the events
        for s_ in seqs:
            if s_:
                out.append(s_.pop(0))
    pk = np.stack([p for p, _ in out])
    ln = np.array([L for _, L in out], np.uint32)
    ref, rst, rlost, rloss, rinp = _oracle(pk, ln)
    n = len(ln)
    for mode in ("fused", "pipelined"):
        got, st, lost, loss, inp = _gpu(hip, pk, ln, stride, [0, n // 2, n], mode, slots=slots)
        assert st == rst, (mode, st, rst)
        assert sorted(got) == sorted(ref), mode
        for k in ref:
            assert sorted(got[k]) == sorted(ref[k]), (k, mode)
        assert lost == rlost and loss == rloss and inp == rinp, mode


@pytest.mark.parametrize("nev,ev_bytes,mtu", [(160, 1 << 20, 1500), (360, 731 * 16, 80), (100, 2200 * 16, 80)])
def test_interleaved_wide_span_sorts_runs(hip, nev, ev_bytes, mtu):
    """Many events interleaved datagram by datagram: a key's span is wide.  160 x 1 MiB (731
    runs per key over ~117 K positions): the walk wave's position bitmap (32 KiB of LDS per
    wave since round 6).  At MTU 80 (16-byte payloads, 64-byte slots) spans too wide for the
    bitmap: 360 events of 731 datagrams (~263 K positions) sort their runs with the bitonic
    wave sort in LDS; 100 events of 2200 datagrams (more than 2048 runs per key) in global
    memory."""
    mp = O.max_pld_len(mtu)
    stride = (36 + mp + 15) // 16 * 16
    pks, lns = [], []
    for k in range(nev):
        ev = np.random.default_rng(1100 + k).integers(0, 256, ev_bytes, dtype=np.uint8)
        pk, ln = O.segment_event(ev, 300 + k, 4321, 1, 2, 2, mp, stride)
        pks.append(pk)
        lns.append(ln)
    pk = np.stack(pks).transpose(1, 0, 2).reshape(-1, pks[0].shape[1])   # round robin over the events
    ln = np.stack(lns).T.reshape(-1)
    ref, rst, rlost, rloss, rinp = _oracle(pk, ln)
    n = len(ln)
    # one batch: the whole span in one walk (a cut would leave each batch's span narrow enough)
    got, st, lost, loss, inp = _gpu(hip, pk, ln, stride, [0, n], "fused", arena=nev * ev_bytes + (8 << 20),
                                    slots=1024 if nev <= 512 else 2048)
    assert st == rst, (st, rst)
    assert sorted(got) == sorted(ref) and len(ref) == nev
    for k in ref:
        assert sorted(got[k]) == sorted(ref[k]), k
    assert lost == rlost and loss == rloss and inp == rinp


def test_reference_order_in_a_replayed_graph(hip):
    """Reference-order launches captured in a HIP graph and replayed: the key pass's run
    filing holds no memset node (its counters are reset by the kernels that use them, a
    captured hipMemsetAsync breaks replays -- DESIGN.md 4.4), and every replay gives the
    oracle's events."""
    import torch
    from e2sar_amd import sar

    rnd = random.Random(5)
    mp = O.max_pld_len(1500)
    stride = (36 + mp + 15) // 16 * 16
    seqs = []
    for k in range(8):
        ev = np.random.default_rng(900 + k).integers(0, 256, 150_000 + 7_777 * k, dtype=np.uint8)
        pk, ln = O.segment_event(ev, 40 + k, 4321, 1, 2, 2, mp, stride)
        order = list(range(len(ln)))
        if k % 3 == 1:
            rnd.shuffle(order)                        # offset 0 anywhere: late offset-0 rules apply
        seqs.append([(pk[i], int(ln[i])) for i in order])
    out = []
    while any(seqs):
        s = rnd.choice([s for s in seqs if s])
        out.append(s.pop(0))
    pk = np.stack([p for p, _ in out])
    ln = np.array([L for _, L in out], np.uint32)
    ref, _, _, _, _ = _oracle(pk, ln)
    n = len(ln)
    dpk = torch.from_numpy(np.ascontiguousarray(pk).reshape(-1)).to(hip.torch_device)
    dln = torch.from_numpy(ln.view(np.int32).copy()).to(hip.torch_device)
    R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=256, queue_capacity=1024, lost_capacity=1024,
                              arena_bytes=64 << 20, flags=_flag())

    def body(stream):
        R.recycle(force=True, stream=stream)
        R.reassemble(dpk, stride, dln, n, stream=stream, now_ms=100)

    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):
        body(cap)                                     # eager first: grows the sort scratch
    torch.cuda.synchronize()
    first = {}
    for rec in R.poll():
        first.setdefault((rec.eventNum, rec.dataId), []).append((R.event_bytes(rec), rec.numFragments))
    assert sorted(first) == sorted(ref)
    for k in ref:
        assert sorted(first[k]) == sorted(ref[k]), k                 # bytes and numFragments
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=cap):
        body(cap)
    for replay in range(3):
        graph.replay()
        torch.cuda.synchronize()
        got = {}
        for rec in R.poll():
            got.setdefault((rec.eventNum, rec.dataId), []).append((R.event_bytes(rec), rec.numFragments))
        assert sorted(got) == sorted(ref), f"replay {replay}"
        for k in ref:
            assert sorted(got[k]) == sorted(ref[k]), (k, replay)
