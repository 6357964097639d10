"""One reassembler driven from two HIP streams at once, and a bench-scale graph round trip.

Config 4 at N > 1 (e2sar_amd.dist.SpreadPipeline) reassembles ONE event table from two
streams concurrently: the in-place fused ``reas_kernel`` of the batch that just landed on
the caller's stream, and ``reas_classify`` + ``reas_scatter`` of the datagrams the exchange
brought (streaming loads, ``set_cold(True)``) on the receive stream -- with fragments of
the same events, offset-0 fragments included, on both sides.  The reference never shares an
in-progress event between receivers (each receive thread owns its map,
e2sarDPReassembler.hpp:223-229); this build does, through the device table's claim/publish
protocol (sar_kernels.hip ``find_or_create``) and per-run atomic accumulators.  The first
test runs exactly that split with both launches in flight together (checked with HIP event
timestamps) and compares events, bytes and every counter with the oracle's reassembly of
the same datagrams in stream order.

The second test is the bench's verified step at bench scale: 1024 x 1 MiB events at MTU
1500 through five 205-event ``seg_kernel`` + ``reas_kernel`` launches per step, four steps
per HIP graph, replayed; every event's bytes and every counter are checked after every
replay.  (Round 4's lookup-first table protocol lost about one event in 4000 there -- a
rate the suite's largest reassembly, 96 events, could not see.)
"""
import numpy as np
import pytest

import oracle_ffi as O

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    return torch


def _source(ctx, n_ev, nbytes, seed):
    torch = _torch()
    g = torch.Generator(device=ctx.torch_device)
    g.manual_seed(seed)
    ev_stride = (nbytes + 255) // 256 * 256
    return torch.randint(0, 256, (n_ev, ev_stride), dtype=torch.uint8, device=ctx.torch_device, generator=g)


def _segment(ctx, src, nbytes, mtu, first_event=0):
    from e2sar_amd import sar
    seg = sar.DeviceSegmenter(ctx, mtu=mtu, lb_hdr_version=2)
    n_ev = src.shape[0]
    plan = seg.plan([(src[i].data_ptr(), nbytes, first_event + i, 4321, 1 + i, (1 << 48) + i) for i in range(n_ev)])
    pk, ln = seg.alloc_packets(plan.total_packets)
    seg.segment(plan, pk, ln)
    return seg, plan, pk, ln


def _oracle_stats(pk, ln, n, stride):
    """The oracle's reassembly of datagrams [0, n) in stream order: stats, event keys, frags."""
    hp = pk[: n * stride].view(n, stride).cpu().numpy()
    hl = ln[:n].cpu().numpy().astype(np.uint32)
    r = O.Reassembler(True, 1 << 20)
    r.push_batch(hp, hl)
    frags = {(e, d): f for _b, e, d, f in r.pop_all_frags()}
    return r.stats(), frags


def _split_sides(n_ev, npk, seed):
    """Side of every datagram (True = the fused in-place side A): offset-0 fragments of even
    events on A and of odd events on B; the others in random runs of 1..40 datagrams."""
    rng = np.random.default_rng(seed)
    side = np.zeros(n_ev * npk, bool)
    for e in range(n_ev):
        j, cur = 0, bool(rng.integers(0, 2))
        while j < npk:
            run = int(rng.integers(1, 41))
            side[e * npk + j: e * npk + min(npk, j + run)] = cur
            cur = not cur
            j += run
        side[e * npk] = (e % 2 == 0)
    return side


@pytest.mark.parametrize("mtu,n_ev,a_first", [(1500, 160, True), (1500, 160, False), (9000, 160, True)])
def test_two_streams_one_reassembler(hip, mtu, n_ev, a_first):
    torch = _torch()
    from e2sar_amd import sar
    B = 1 << 20
    src = _source(hip, n_ev, B, 0xC0C0 + mtu + int(a_first))
    seg, plan, pk, ln = _segment(hip, src, B, mtu)
    stride, n = seg.stride, plan.total_packets
    npk = n // n_ev
    side = _split_sides(n_ev, npk, mtu + int(a_first))
    ia = torch.from_numpy(np.nonzero(side)[0]).to(hip.torch_device)
    ib = torch.from_numpy(np.nonzero(~side)[0]).to(hip.torch_device)
    rows = pk[: n * stride].view(n, stride)
    apk, aln = rows.index_select(0, ia).contiguous().view(-1), ln[:n].index_select(0, ia).contiguous()
    bpk, bln = rows.index_select(0, ib).contiguous().view(-1), ln[:n].index_select(0, ib).contiguous()
    na, nb = int(ia.numel()), int(ib.numel())
    assert na and nb
    ost, ofr = _oracle_stats(pk, ln, n, stride)
    overlapped = []
    # the HIP runtime maps streams onto a few hardware queues; two streams that share one run
    # one after the other, so each attempt takes a new pair (the second at high priority) and
    # the test needs one attempt whose launches overlapped -- every attempt is checked in full
    for attempt in range(4):
        R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=4096, queue_capacity=2 * n_ev,
                                  arena_bytes=n_ev * B + 4096)
        R.set_cold(True)                               # what the spread leg sets for received datagrams
        work = R.alloc_work(nb)
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream(priority=-1 if attempt % 2 else 0)
        ref = torch.cuda.Event(enable_timing=True)
        ev = {k: torch.cuda.Event(enable_timing=True) for k in ("a0", "a1", "b0", "b1")}
        torch.cuda.synchronize()
        # a gate: both streams wait behind a spin kernel, so every launch below is queued
        # when it opens and the two sides start together
        torch.cuda._sleep(20_000_000)
        ref.record()
        sa.wait_event(ref)
        sb.wait_event(ref)

        def side_a():
            ev["a0"].record(sa)
            R.reassemble(apk, stride, aln, na, stream=sa)          # SpreadPipeline.land
            ev["a1"].record(sa)

        def side_b():
            ev["b0"].record(sb)
            R.classify(bpk, stride, bln, nb, work, stream=sb)     # SpreadPipeline._reassemble_received
            R.scatter(bpk, stride, nb, work, stream=sb)
            ev["b1"].record(sb)

        for f in ((side_a, side_b) if a_first else (side_b, side_a)):
            f()
        torch.cuda.synchronize()
        t = {k: ref.elapsed_time(e) for k, e in ev.items()}
        # the two launches were in flight together: each started before the other ended
        overlapped.append((t["a0"] < t["b1"] and t["b0"] < t["a1"], t))

        recs = R.poll()
        st = R.stats()
        assert {(r.eventNum, r.dataId) for r in recs} == set(ofr)
        for f in ("eventSuccess", "totalPackets", "totalBytes", "badHeaderDiscards", "dataErrCnt",
                  "enqueueLoss", "reassemblyLoss"):
            assert getattr(st, f) == ost[f], (f, getattr(st, f), ost[f])
        assert st.inProgress == ost["inProgress"] == 0
        arena = R.arena_tensor()
        for r in recs:
            assert r.bytes == B and r.numFragments == ofr[(r.eventNum, r.dataId)]
            assert torch.equal(arena[r.arenaOffset: r.arenaOffset + B], src[r.eventNum, :B]), r.eventNum
        R.close()
        if overlapped[-1][0]:
            break
    print("two-stream timings (ms after the gate):", overlapped)
    assert overlapped[-1][0], f"the two streams never ran together: {overlapped}"


@pytest.mark.parametrize("fold", [False, True])
def test_bench_scale_graph_roundtrip(hip, fold):
    """bench.py's headline step (config 2) as a suite test: 1024 x 1 MiB at MTU 1500, five
    205-event batches, four steps per captured graph, three replays, all verified.  fold:
    the step's recycle runs inside its first segmentation launch
    (e2sar_hip_segment_batch_recycle), as bench.py's default step does."""
    torch = _torch()
    from e2sar_amd import sar
    B, E, BATCH, STEPS, REPLAYS = 1 << 20, 1024, 205, 4, 3
    src = _source(hip, E, B, 0xE25A2)
    seg = sar.DeviceSegmenter(hip, mtu=1500, lb_hdr_version=2)
    stride, npk = seg.stride, sar.num_packets(B, seg.max_pld)
    plans = [seg.plan([(src[i].data_ptr(), B, i, 4321, 1 + (i * 0x9E37) % 65535, (1 << 48) + i)
                       for i in range(b0, min(E, b0 + BATCH))]) for b0 in range(0, E, BATCH)]
    assert len(plans) == 5
    pk, ln = seg.alloc_packets(max(p.total_packets for p in plans))
    R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=8192, queue_capacity=E + 64,
                              lost_capacity=1024, arena_bytes=E * B + 4096)

    def step():
        if not fold:
            R.recycle(force=True)
        for k, p in enumerate(plans):
            if k == 0 and fold:
                seg.segment(p, pk, ln, recycle=R, force=True)
            else:
                seg.segment(p, pk, ln)
            R.reassemble(pk, stride, ln, p.total_packets)

    # the oracle's counters for one event's datagrams (the stream is E such events in order)
    p1 = seg.plan([(src[0].data_ptr(), B, 0, 4321, 1, 1 << 48)])
    pk1, ln1 = seg.alloc_packets(p1.total_packets)
    seg.segment(p1, pk1, ln1)
    ost, ofr = _oracle_stats(pk1, ln1, p1.total_packets, stride)
    assert ost["eventSuccess"] == 1 and ofr[(0, 4321)] == npk

    step()                                        # warm up (and the first, eager, check)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(graph, stream=cap):
        for _ in range(STEPS):
            step()
    torch.cuda.synchronize()
    R.poll()
    arena = R.arena_tensor()
    for rep in range(REPLAYS):
        before = R.stats()
        graph.replay()
        torch.cuda.synchronize()
        recs = R.poll()
        st = R.stats()
        assert len(recs) == E, (rep, len(recs), st.inProgress)
        assert sorted(r.eventNum for r in recs) == list(range(E))
        for f in ("eventSuccess", "totalPackets", "totalBytes"):
            assert getattr(st, f) - getattr(before, f) == STEPS * E * ost[f], (rep, f)
        for f in ("badHeaderDiscards", "dataErrCnt", "enqueueLoss", "reassemblyLoss"):
            assert getattr(st, f) == 0, (rep, f, getattr(st, f))
        assert st.inProgress == 0
        bad = [r.eventNum for r in recs
               if r.numFragments != npk or r.bytes != B
               or not torch.equal(arena[r.arenaOffset: r.arenaOffset + B], src[r.eventNum, :B])]
        assert not bad, (rep, bad[:8])


def test_forget_stream_then_destroy(hip):
    """e2sar_hip_reas_forget_stream: reassemble on a stream of our own (reference-order mode,
    so the stream gets internal scratch), forget it, destroy it, then launch on a fresh
    stream (HIP may reuse the handle) and snapshot -- every event and counter as the oracle's."""
    import ctypes as C
    torch = _torch()
    from e2sar_amd import _capi, sar
    from e2sar_amd._capi import check, lib
    B, n_ev = 100_000, 6
    src = _source(hip, n_ev, B, 0xF0F0)
    seg, plan, pk, ln = _segment(hip, src, B, 1500)
    stride, n = seg.stride, plan.total_packets
    half = n // 2
    R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=64, arena_bytes=n_ev * B + 4096,
                              flags=_capi.REAS_REFERENCE_ORDER)
    torch.cuda.synchronize()
    s1 = C.c_void_p()
    check(lib().e2sar_hip_stream_create(0, C.byref(s1)))
    check(lib().e2sar_hip_reassemble_batch(R.handle, C.c_void_p(pk.data_ptr()), stride, C.c_void_p(ln.data_ptr()),
                                           half, 0, s1))
    check(lib().e2sar_hip_reas_forget_stream(R.handle, s1))          # waits for s1, drops its scratch
    check(lib().e2sar_hip_stream_destroy(s1))
    s2 = C.c_void_p()
    check(lib().e2sar_hip_stream_create(0, C.byref(s2)))
    check(lib().e2sar_hip_reassemble_batch(R.handle, C.c_void_p(pk[half * stride:].data_ptr()), stride,
                                           C.c_void_p(ln[half:].data_ptr()), n - half, 0, s2))
    recs = R.poll()                                                 # waits for s2 (and not for s1)
    st = R.stats()
    ost, ofr = _oracle_stats(pk, ln, n, stride)
    assert {(r.eventNum, r.dataId) for r in recs} == set(ofr)
    for f in ("eventSuccess", "totalPackets", "totalBytes", "badHeaderDiscards", "dataErrCnt"):
        assert getattr(st, f) == ost[f], f
    arena = R.arena_tensor()
    for r in recs:
        assert torch.equal(arena[r.arenaOffset: r.arenaOffset + B], src[r.eventNum, :B])
    ts = torch.cuda.Stream()                                        # the Python wrapper
    R.gc(now_ms=1, timeout_ms=1 << 40, stream=ts)
    R.forget_stream(ts)
    check(lib().e2sar_hip_reas_forget_stream(R.handle, s2))
    check(lib().e2sar_hip_stream_destroy(s2))
    assert R.stats().eventSuccess == ost["eventSuccess"]


def test_context_destroyed_before_its_reassembler(hip):
    """A garbage collector tearing down a reference cycle destroys a Context and the
    DeviceReassembler made on it in either order; the reassembler holds a reference on the
    context (capi.cpp), so reas_destroy never reads a freed context (it once set the device
    from one: 'invalid device ordinal' on the next HIP call of the process)."""
    torch = _torch()
    from e2sar_amd import sar
    for first in ("ctx", "reas"):
        ctx = sar.Context(0)
        R = sar.DeviceReassembler(ctx, with_lb_header=True, table_slots=64, arena_bytes=1 << 20)
        R.recycle(force=True)
        torch.cuda.synchronize()
        if first == "ctx":
            ctx.close()
            R.close()
        else:
            R.close()
            ctx.close()
        x = torch.full((64,), 7, dtype=torch.int32, device=hip.torch_device)
        assert torch.equal(x, x.clone())                          # the process is still healthy


def test_segment_batch_recycle_preconditions(hip):
    """e2sar_hip_segment_batch_recycle without force refuses as e2sar_hip_reas_recycle does
    (completed records not yet polled), and once polled it segments and recycles in one launch:
    the arena and table are empty again and the next reassembly starts from offset 0."""
    torch = _torch()
    from e2sar_amd import sar
    B, n_ev = 100_000, 4
    src = _source(hip, n_ev, B, 0xACE)
    seg, plan, pk, ln = _segment(hip, src, B, 1500)
    stride, n = seg.stride, plan.total_packets
    R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=64, arena_bytes=n_ev * B + 4096)
    R.reassemble(pk, stride, ln, n)
    pk2, ln2 = seg.alloc_packets(n)
    from e2sar_amd._capi import E2SARHipError
    with pytest.raises(E2SARHipError):
        seg.segment(plan, pk2, ln2, recycle=R, force=False)      # records not polled yet
    first = R.poll()
    assert len(first) == n_ev
    st = R.stats()
    assert st.arenaUsed > 0 and st.tableUsed == n_ev
    seg.segment(plan, pk2, ln2, recycle=R, force=False)
    torch.cuda.synchronize()
    st = R.stats()
    assert st.arenaUsed == 0 and st.tableUsed == 0 and st.inProgress == 0
    assert torch.equal(ln2[:n], ln[:n])
    a = pk[: n * stride].view(n, stride).cpu().numpy()
    b = pk2[: n * stride].view(n, stride).cpu().numpy()
    L = ln[:n].cpu().numpy()
    assert all(np.array_equal(a[k, : L[k]], b[k, : L[k]]) for k in range(n))
    R.reassemble(pk2, stride, ln2, n)
    recs = R.poll()
    assert sorted(r.eventNum for r in recs) == sorted(r.eventNum for r in first)
    assert min(r.arenaOffset for r in recs) == 0
    arena = R.arena_tensor()
    for r in recs:
        assert torch.equal(arena[r.arenaOffset: r.arenaOffset + B], src[r.eventNum, :B])
