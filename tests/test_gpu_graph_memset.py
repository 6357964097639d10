"""Captured memsets and graph replays.

On this ROCm a hipMemsetAsync node of 64 bytes or more captured into a HIP graph writes
garbage from the second replay on (tools/graph_memset_probe.py); 4- and 8-byte nodes replay
clean.  The first test below keeps the round-1 shape (4- and 8-byte nodes); the second pins
that e2sar_hip_memset_d, a fill kernel, replays exactly.

A captured 4-byte hipMemsetAsync followed by the reassembly kernels, replayed.

Round 1 saw "the next kernel" fault on the second replay of a step graph that held
4-byte memset nodes (e2sar_hip_reas_reset_stats, since replaced by zero_words_kernel).
The memset targets live in the control block, which compaction never replaces (it swaps
only the slot table and the arena), so a stale captured pointer is ruled out (DESIGN.md
4.4).  This test rebuilds the suspected shape on its own: memset nodes of 4 bytes at an
address 12 mod 16 (where errorFlags sits) and 8 bytes at 0 mod 16, then recycle and
reassemble, captured once and replayed three times; guard bytes around each target
must survive and every replay must reassemble every event.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O

pytestmark = pytest.mark.gpu


def test_captured_small_memsets_then_reassembly_replay(hip):
    import torch
    from e2sar_amd import sar

    hiprt = C.CDLL("libamdhip64.so")
    hiprt.hipMemsetAsync.restype = C.c_int
    hiprt.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]

    mp = O.max_pld_len(1500)
    stride = (36 + mp + 15) // 16 * 16
    evs = [np.random.default_rng(40 + k).integers(0, 256, 20000 + 999 * k, dtype=np.uint8) for k in range(5)]
    pks, lns = [], []
    for k, e in enumerate(evs):
        p, l = O.segment_event(e, k, 4321, 1 + k, 9, 2, mp, stride)
        pks.append(p)
        lns.append(l)
    pk = np.concatenate(pks)
    ln = np.concatenate(lns)
    n = len(ln)
    dpk = torch.from_numpy(pk.reshape(-1).copy()).to(hip.torch_device)
    dln = torch.from_numpy(ln.view(np.int32).copy()).to(hip.torch_device)
    R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=64, arena_bytes=1 << 20)
    guard = torch.full((256,), 0xAB, dtype=torch.uint8, device=hip.torch_device)
    base = guard.data_ptr()
    assert base % 256 == 0

    def body(stream):
        h = C.c_void_p(int(stream.cuda_stream))
        assert hiprt.hipMemsetAsync(C.c_void_p(base + 172), 0, 4, h) == 0      # 12 mod 16, like errorFlags
        assert hiprt.hipMemsetAsync(C.c_void_p(base + 160), 0, 8, h) == 0      # 0 mod 16, like nCompleted/nLost
        R.recycle(force=True, stream=stream)
        R.reassemble(dpk, stride, dln, n, stream=stream)

    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):
        body(cap)
    torch.cuda.synchronize()
    R.poll()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=cap):
        body(cap)
    expect = np.full(256, 0xAB, np.uint8)
    expect[160:168] = 0
    expect[172:176] = 0
    for replay in range(3):
        guard.fill_(0xAB)
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(guard.cpu().numpy(), expect, err_msg=f"replay {replay}")
        got = {r.eventNum: R.event_bytes(r) for r in R.poll()}
        assert sorted(got) == list(range(5)), f"replay {replay}"
        assert all(got[k] == evs[k].tobytes() for k in range(5)), f"replay {replay}"


@pytest.mark.parametrize("value", [0, 0xA5])
def test_memset_d_eager_and_in_a_replayed_graph(value):
    """e2sar_hip_memset_d is a fill kernel: exact bytes at any alignment and size, eagerly and
    captured in a HIP graph replayed three times (hipMemsetAsync nodes of 64 bytes and more
    write garbage from the second replay on, tools/graph_memset_probe.py)."""
    import torch
    from e2sar_amd import sar
    from e2sar_amd._capi import lib

    cap = torch.cuda.Stream()
    ctx = sar.Context(0, stream=cap)
    buf = torch.zeros(1 << 20, dtype=torch.uint8, device=ctx.torch_device)
    base = buf.data_ptr()
    cases = [(0, 1), (3, 5), (1, 16), (7, 64), (16, 4096), (5, 4100), (9, 100_003), (0, 1 << 19)]

    def body():
        for off, n in cases:
            assert lib().e2sar_hip_memset_d(ctx.handle, C.c_void_p(base + 1024 + off * 3 + (n if n < 4096 else 0)),
                                            value, n) == 0

    def expected():
        e = np.full(buf.numel(), 0x11, np.uint8)
        for off, n in cases:
            a = 1024 + off * 3 + (n if n < 4096 else 0)
            e[a:a + n] = value
        return e

    buf.fill_(0x11)
    torch.cuda.synchronize()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):
        body()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(buf.cpu().numpy(), expected())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=cap):
        body()
    for replay in range(3):
        buf.fill_(0x11)
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(buf.cpu().numpy(), expected(), err_msg=f"replay {replay}")
    ctx.close()
