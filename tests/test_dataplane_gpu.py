"""Reference-shaped data-plane tests through e2sar_py (C++ facade -> C ABI -> gfx950).

Mirrors test/e2sar_seg_test.cpp (DPSegTest1-4), test/e2sar_reas_test.cpp (DPReasTest1-4)
and test/py_test/test_b2b_DP.py: UDP loopback on 127.0.0.1, useCP off, the Reassembler
expecting the LB header the missing load balancer would have stripped.  Datagrams
captured on a plain socket are compared bit-for-bit with the oracle, taking the
per-event LB tick and entropy (random by design in the reference) from the datagram.
"""
import os
import socket
import threading
import time

import numpy as np
import pytest

import oracle_ffi as O

pytestmark = pytest.mark.gpu

DP = "127.0.0.1"
DATA_ID = 0x0505
EVENTSRC_ID = 0x11223344
SEND_STR = b"THIS IS A VERY LONG EVENT MESSAGE WE WANT TO SEND EVERY 1 SECONDS."   # 67 bytes
_port = [21000]


def next_port(span=1):
    p = _port[0]
    _port[0] += max(span, 8)
    return p


@pytest.fixture(scope="module")
def E():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no GPU is visible")
    from e2sar_amd import e2sar_py
    return e2sar_py


def make_seg(E, port, mtu=1500, sockets=4, ver=2, rate=-1.0, data_id=DATA_ID):
    uri = E.EjfatURI(f"ejfat://useless@192.168.100.1:9875/lb/1?sync=192.168.0.1:12345&data={DP}:{port}",
                     E.EjfatURI.TokenType.instance)
    f = E.DataPlane.Segmenter.SegmenterFlags()
    f.useCP = False
    f.mtu = mtu
    f.numSendSockets = sockets
    f.lbHdrVersion = ver
    f.rateGbps = rate
    return E.DataPlane.Segmenter(uri, data_id, EVENTSRC_ID, f)


def make_reas(E, port, threads=1, with_lb=True, timeout_ms=500, port_range=-1):
    uri = E.EjfatURI(f"ejfat://useless@192.168.100.1:9875/lb/1?sync=192.168.0.1:12345&data={DP}",
                     E.EjfatURI.TokenType.instance)
    f = E.DataPlane.Reassembler.ReassemblerFlags()
    f.useCP = False
    f.withLBHeader = with_lb
    f.eventTimeout_ms = timeout_ms
    f.portRange = port_range
    f.rcvSocketBufSize = 4 * 1024 * 1024
    f.arenaBytes = 256 << 20
    return E.DataPlane.Reassembler(uri, E.IPAddress.from_string(DP), port, threads, f)


def ok(res):
    assert not res.has_error(), res.error()
    assert res.value() == 0


def capture(port, n, timeout=5.0):
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    s.bind((DP, port))
    s.settimeout(timeout)
    out = []

    def run():
        try:
            while len(out) < n:
                out.append(s.recv(16384))
        except socket.timeout:
            pass
        s.close()

    t = threading.Thread(target=run)
    t.start()
    return t, out


def check_against_oracle(dgrams, payloads, mtu, ver, data_id, first_evnum):
    """Every captured datagram == the oracle's, with tick/entropy taken from the datagram."""
    mp = O.max_pld_len(mtu)
    by_ev = {}
    for d in dgrams:
        okv, did, off, blen, ev, _ = O.re_parse(d[16:36])
        assert okv and did == data_id
        by_ev.setdefault(ev, []).append(d)
    assert sorted(by_ev) == list(range(first_evnum, first_evnum + len(payloads)))
    for k, p in enumerate(payloads):
        got = sorted(by_ev[first_evnum + k], key=lambda d: int.from_bytes(d[20:24], "big"))
        tick = int.from_bytes(got[0][8:16], "big")
        ent = int.from_bytes(got[0][6:8], "big")
        pk, ln = O.segment_event(np.frombuffer(p, np.uint8), first_evnum + k, data_id, ent, tick, ver, mp)
        assert len(got) == len(ln)
        for j, d in enumerate(got):
            assert d == pk[j, : int(ln[j])].tobytes(), f"event {k} datagram {j} differs"


# ------------------------------- Segmenter ---------------------------------------

@pytest.mark.parametrize("mtu,per_event", [(1500, 1), (104, 2)])
def test_dpsegtest1_2_send_event(E, mtu, per_event):
    # DPSegTest1 (msgCnt 5) / DPSegTest2-3 (MTU 104 -> msgCnt 10)
    port = next_port()
    t, got = capture(port, 5 * per_event)
    seg = make_seg(E, port, mtu=mtu)
    ok(seg.OpenAndStart())
    assert seg.getSendStats().msgCnt == 0
    for _ in range(5):
        ok(seg.sendEvent(SEND_STR, len(SEND_STR)))
    st = seg.getSendStats()
    assert st.msgCnt == 5 * per_event and st.errCnt == 0
    t.join()
    seg.stopThreads()
    assert len(got) == 5 * per_event
    check_against_oracle(got, [SEND_STR] * 5, mtu, 2, DATA_ID, 0)


def test_dpsegtest4_queue_callbacks_v3(E):
    port = next_port()
    t, got = capture(port, 10)
    seg = make_seg(E, port, mtu=104, ver=3)
    ok(seg.OpenAndStart())
    fired = []
    for i in range(5):
        ok(seg.addToSendQueue(SEND_STR, len(SEND_STR), 0, 0, 0, lambda a: fired.append(a), i))
    seg.stopThreads()            # drains the queue first (hpp:537-552)
    t.join()
    assert seg.getSendStats().msgCnt == 10
    assert sorted(fired) == [0, 1, 2, 3, 4]
    check_against_oracle(got, [SEND_STR] * 5, 104, 3, DATA_ID, 0)


def test_event_numbering_and_overrides(E):
    # sendEvent(_eventNum != 0) resets the counter (cpp:905-906); _dataId overrides (cpp:913)
    port = next_port()
    t, got = capture(port, 3)
    seg = make_seg(E, port)
    ok(seg.OpenAndStart())
    ok(seg.sendEvent(SEND_STR, len(SEND_STR), 100, 0, 0))
    ok(seg.sendEvent(SEND_STR, len(SEND_STR), 0, 77, 0x1234))
    ok(seg.sendEvent(SEND_STR, len(SEND_STR)))
    t.join()
    seg.stopThreads()
    evs = sorted((O.re_parse(d[16:36])[4], O.re_parse(d[16:36])[1], int.from_bytes(d[6:8], "big")) for d in got)
    assert evs[0][:2] == (100, DATA_ID) and evs[1] == (101, 77, 0x1234) and evs[2][:2] == (102, DATA_ID)


def test_ticks_as_re_event_num(E):
    # ticksAsREEventNum: the RE eventNum carries the LB tick (e2sarDPSegmenter.cpp:723-724)
    port = next_port()
    t, got = capture(port, 2)
    f = E.DataPlane.Segmenter.SegmenterFlags()
    f.useCP = False
    f.mtu = 1500
    f.numSendSockets = 1
    f.ticksAsREEventNum = True
    uri = E.EjfatURI(f"ejfat://useless@192.168.100.1:9875/lb/1?sync=192.168.0.1:12345&data={DP}:{port}",
                     E.EjfatURI.TokenType.instance)
    seg = E.DataPlane.Segmenter(uri, DATA_ID, EVENTSRC_ID, f)
    ok(seg.OpenAndStart())
    ok(seg.sendEvent(SEND_STR, len(SEND_STR), 5, 0, 0))
    ok(seg.sendEvent(SEND_STR, len(SEND_STR), 6, 0, 0))
    t.join()
    seg.stopThreads()
    assert len(got) == 2
    for d in got:
        tick = int.from_bytes(d[8:16], "big")
        assert O.re_parse(d[16:36])[4] == tick and tick > (1 << 40)   # a microsecond clock, not 5 / 6


def test_segmenter_sanity_checks(E):
    uri = E.EjfatURI(f"ejfat://u@1.2.3.4:1/lb/1?data={DP}:{next_port()}")
    f = E.DataPlane.Segmenter.SegmenterFlags()
    with pytest.raises(E.E2SARException):        # useCP without a sync address (hpp:306-307)
        E.DataPlane.Segmenter(uri, 1, 2, f)
    f.useCP = False
    f.mtu = 9001
    with pytest.raises(E.E2SARException):        # MTU > 9000 (hpp:310-311)
        E.DataPlane.Segmenter(uri, 1, 2, f)
    f.mtu = 64
    with pytest.raises(E.E2SARException):        # MTU <= headers (hpp:315-316)
        E.DataPlane.Segmenter(uri, 1, 2, f)
    f.mtu = 1500
    f.lbHdrVersion = 4
    with pytest.raises(E.E2SARException):        # cpp:52-53
        E.DataPlane.Segmenter(uri, 1, 2, f)


# ------------------------------- Reassembler -------------------------------------

@pytest.mark.parametrize("mtu,per_event", [(1500, 1), (80, 5)])
def test_dpreastest1_2_loopback(E, mtu, per_event):
    port = next_port()
    reas = make_reas(E, port)
    ok(reas.OpenAndStart())
    seg = make_seg(E, port, mtu=mtu)
    ok(seg.OpenAndStart())
    for _ in range(5):
        ok(seg.sendEvent(SEND_STR, len(SEND_STR)))
    assert seg.getSendStats().msgCnt == 5 * per_event
    got = []
    for _ in range(5):
        n, data, ev, did = reas.recvEventBytes(2000)
        assert n == len(SEND_STR) and data == SEND_STR and did == DATA_ID
        got.append(ev)
    assert sorted(got) == [0, 1, 2, 3, 4]
    st = reas.getStats()
    assert st.eventSuccess == 5 and st.enqueueLoss == 0 and st.reassemblyLoss == 0
    assert st.totalPackets == 5 * per_event and st.badHeaderDiscards == 0
    assert reas.get_LostEvent() == ()
    seg.stopThreads()
    reas.stopThreads()


def test_dpreastest3_port_ranges(E):
    base = 19522
    cases = [(1, -1, 0, (base, base)), (4, -1, 2, (base, base + 3)), (7, -1, 3, (base, base + 7)),
             (1, 10, 10, (base, base + 1023)), (1, 1, 1, (base, base + 1))]
    for threads, pr, want_pr, ports in cases:
        r = make_reas(E, base, threads=threads, port_range=pr)
        assert r.get_numRecvThreads() == threads
        assert r.get_portRange() == want_pr
        assert r.get_recvPorts() == ports
        del r


def test_dpreastest4_many_senders_fd_stats(E):
    # 4 Segmenters -> 4 ports -> 1 receive thread; 20 events; per-port counts after stop
    port = next_port(8)
    reas = make_reas(E, port, threads=1, port_range=2)
    ok(reas.OpenAndStart())
    segs = [make_seg(E, port + i, data_id=DATA_ID + i) for i in range(4)]
    for s in segs:
        ok(s.OpenAndStart())
    for k in range(5):
        for s in segs:
            ok(s.sendEvent(SEND_STR, len(SEND_STR)))
    got = 0
    while got < 20:
        n, data, ev, did = reas.recvEventBytes(2000)
        assert n == len(SEND_STR) and data == SEND_STR
        got += 1
    st = reas.getStats()
    assert st.eventSuccess == 20 and st.enqueueLoss == 0 and st.reassemblyLoss == 0
    assert reas.get_FDStats().has_error()          # only after the threads stop
    for s in segs:
        s.stopThreads()
    reas.stopThreads()
    fd = dict(reas.get_FDStats().value())
    assert sorted(fd) == [port, port + 1, port + 2, port + 3] and all(v == 5 for v in fd.values())


def test_lost_event_after_timeout(E):
    # two of five fragments of event 9 never arrive: GC logs it (cpp:252-274, hpp:262-279)
    port = next_port()
    reas = make_reas(E, port, timeout_ms=200)
    ok(reas.OpenAndStart())
    mp = O.max_pld_len(80)
    pk, ln = O.segment_event(np.frombuffer(SEND_STR, np.uint8), 9, 33, 5, 6, 2, mp)
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    for j in (0, 2, 4):
        s.sendto(pk[j, : int(ln[j])].tobytes(), (DP, port))
    s.sendto(b"\x00" * 40, (DP, port))             # bad RE header
    deadline = time.time() + 5
    lost = ()
    while time.time() < deadline and lost == ():
        time.sleep(0.1)
        lost = reas.get_LostEvent()
    assert lost == (9, 33, 3)
    st = reas.getStats()
    assert st.reassemblyLoss == 1 and st.eventSuccess == 0 and st.badHeaderDiscards == 1
    assert st.totalPackets == 4
    reas.stopThreads()


# ------------------------------- back to back (test_b2b_DP.py) -------------------

def test_b2b_send_bytes_recv_bytes(E):
    port = next_port()
    reas = make_reas(E, port)
    ok(reas.OpenAndStart())
    seg = make_seg(E, port)
    ok(seg.OpenAndStart())
    msg = SEND_STR[:65]
    ok(seg.sendEvent(msg, len(msg)))
    assert seg.getSendStats().msgCnt == 1
    n, data, ev, did = reas.recvEventBytes(2000)
    assert n == len(msg) and data == msg and did == DATA_ID
    reas.stopThreads()
    seg.stopThreads()


def test_b2b_send_numpy_get_numpy(E):
    port = next_port()
    reas = make_reas(E, port)
    ok(reas.OpenAndStart())
    seg = make_seg(E, port, rate=2.0)
    ok(seg.OpenAndStart())
    arr = np.random.default_rng(1).random((100, 100, 50), dtype=np.float32)   # 2,000,000 bytes
    ok(seg.sendNumpyArray(arr, arr.nbytes))
    n, out, ev, did = reas.recv1DNumpyArray(np.float32().dtype, 5000)
    assert n == arr.nbytes and did == DATA_ID
    assert np.array_equal(arr.flatten(), out)
    reas.stopThreads()
    seg.stopThreads()


def test_b2b_send_numpy_queue_get_numpy(E):
    port = next_port()
    reas = make_reas(E, port)
    ok(reas.OpenAndStart())
    seg = make_seg(E, port)
    ok(seg.OpenAndStart())
    rows = np.random.default_rng(2).integers(0, 256, (5, 100), dtype=np.uint8)
    done = []
    for i in range(5):
        ok(seg.addNumpyArrayToSendQueue(rows[i], rows[i].nbytes, 0, 0, 0, lambda a: done.append(a), i))
    recv = []
    while len(recv) < 5:
        n, out, ev, did = reas.recv1DNumpyArray(np.uint8().dtype, 3000)
        assert n == 100
        recv.append(out.tobytes())
    seg.stopThreads()
    assert sorted(done) == [0, 1, 2, 3, 4]
    assert sorted(recv) == sorted(r.tobytes() for r in rows)      # order-insensitive (:251-256)
    reas.stopThreads()


def test_b2b_large_events_jumbo(E):
    # 24 x 1 MiB at MTU 9000 through the socket path, paced so loopback does not drop
    port = next_port()
    reas = make_reas(E, port)
    ok(reas.OpenAndStart())
    seg = make_seg(E, port, mtu=9000, rate=4.0)
    ok(seg.OpenAndStart())
    rng = np.random.default_rng(3)
    evs = [rng.integers(0, 256, 1 << 20, dtype=np.uint8) for _ in range(24)]
    for e in evs:
        ok(seg.addNumpyArrayToSendQueue(e, e.nbytes))
    got = {}
    while len(got) < 24:
        n, out, ev, did = reas.recv1DNumpyArray(np.uint8().dtype, 10000)
        assert n == 1 << 20, (n, reas.getStats().reassemblyLoss)
        got[ev] = out
    seg.stopThreads()
    for k, e in enumerate(evs):
        assert np.array_equal(got[k], e)
    assert reas.getStats().eventSuccess == 24
    reas.stopThreads()


@pytest.mark.gpu
def test_e2sar_perf_tool_loopback():
    # the e2sar_perf-shaped tool (tools/e2sar_perf.cpp) end to end over UDP loopback:
    # Segmenter -> seg_kernel -> sendmmsg -> recvmmsg -> reas_kernel -> recvEvent
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "e2sar_perf")
    if not os.path.exists(exe):
        pytest.fail("build/e2sar_perf missing: run make")
    r = subprocess.run([exe, "--loopback", "-l", "100000", "-n", "50", "-m", "9000", "--rate", "2",
                        "--port", "10400"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "50 of 50 events intact" in r.stdout
    assert "eventSuccess=50" in r.stdout and "badHeaderDiscards=0" in r.stdout


@pytest.mark.gpu
def test_sync_thread_frames(E):
    # DPSyncTest1 (test/e2sar_sync_test.cpp:25-64) and the sync half of DPSegTest1
    # (e2sar_seg_test.cpp:83-93), scaled from 1 s to 50 ms periods: with useCP the
    # Segmenter sends a 28-byte SyncHdr (e2sarHeaders.hpp:323-403) to the URI's sync
    # address every syncPeriodMs, starting with a warm-up before any data
    import struct
    sport, dport = next_port(), next_port()
    cap = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    cap.bind((DP, sport))
    cap.settimeout(0.2)
    uri = E.EjfatURI(f"ejfat://useless@192.168.100.1:9875/lb/1?sync={DP}:{sport}&data={DP}:{dport}",
                     E.EjfatURI.TokenType.instance)
    f = E.DataPlane.Segmenter.SegmenterFlags()
    f.useCP = True
    f.syncPeriodMs = 50
    f.warmUpMs = 100
    seg = E.DataPlane.Segmenter(uri, DATA_ID, EVENTSRC_ID, f)
    t0 = time.time_ns()
    ok(seg.OpenAndStart())
    assert time.time_ns() - t0 >= 100_000_000            # the warm-up happens inside OpenAndStart
    time.sleep(0.5)
    seg.stopThreads()
    t1 = time.time_ns()
    st = seg.getSyncStats()
    frames = []
    try:
        while True:
            frames.append(cap.recv(100))
    except socket.timeout:
        pass
    cap.close()
    assert st.errCnt == 0
    assert 9 <= st.msgCnt <= 16, st.msgCnt               # ~0.6 s / 50 ms
    assert len(frames) == st.msgCnt
    prev = (0, 0)
    for fr in frames:
        assert len(fr) == 28
        pre, ver, rsvd, esid, evn, rate, tns = struct.unpack(">2sBBIQIQ", fr)
        assert (pre, ver, rsvd, esid, rate) == (b"LC", 2, 0, EVENTSRC_ID, 1000000)
        assert t0 <= tns <= t1
        assert abs(evn - tns // 1000) < 1000             # eventNumber: the clock in microseconds
        assert (evn, tns) > prev
        prev = (evn, tns)


@pytest.mark.gpu
def test_e2sar_ft_tool_loopback(tmp_path):
    # the e2sar_ft-shaped tool (tools/e2sar_ft.cpp, bin/e2sar_ft.cpp): every file matching
    # the extension becomes one event (mmap -> addToSendQueue -> seg_kernel -> UDP ->
    # reas_kernel -> recvEvent) and is written back as <prefix>_<event>_<dataId><ext>
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "e2sar_ft")
    if not os.path.exists(exe):
        pytest.fail("build/e2sar_ft missing: run make")
    src, out = tmp_path / "in", tmp_path / "out"
    src.mkdir()
    out.mkdir()
    rng = np.random.default_rng(11)
    sizes = [1, 67, 1436, 1437, 100_000, (1 << 20) + 3]
    names = [f"f{k}.dat" for k in range(len(sizes))]
    for n, s in zip(names, sizes):
        (src / n).write_bytes(rng.integers(0, 256, s, dtype=np.uint8).tobytes())
    (src / "skip.txt").write_bytes(b"not sent")
    r = subprocess.run([exe, "--loopback", "-p", str(out), "--port", str(next_port()), "-e", ".dat",
                        "--dataid", "4321", "-m", "9000", str(src)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = sorted(p.name for p in out.iterdir())
    assert got == sorted(f"e2sar_out_{k}_4321.dat" for k in range(len(sizes)))
    for k, n in enumerate(sorted(names)):
        assert (out / f"e2sar_out_{k}_4321.dat").read_bytes() == (src / n).read_bytes(), n


@pytest.mark.gpu
def test_ipv6_loopback(E):
    # dpV6: IPv6 data address from the URI, maxPldLen = mtu - 84 (e2sarHeaders.hpp:415-421),
    # datagrams over ::1 reassembled bit-exactly
    try:
        probe = socket.socket(socket.AF_INET6, socket.SOCK_DGRAM)
        probe.bind(("::1", 0))
        probe.close()
    except OSError:
        pytest.skip("no IPv6 loopback on this host")
    port = next_port()
    uri = E.EjfatURI(f"ejfat://useless@192.168.100.1:9875/lb/1?data=[::1]:{port}", E.EjfatURI.TokenType.instance)
    sf = E.DataPlane.Segmenter.SegmenterFlags()
    sf.useCP = False
    sf.dpV6 = True
    seg = E.DataPlane.Segmenter(uri, DATA_ID, EVENTSRC_ID, sf)
    assert seg.getMaxPldLen() == 1500 - 84
    rf = E.DataPlane.Reassembler.ReassemblerFlags()
    rf.useCP = False
    rf.withLBHeader = True
    rf.arenaBytes = 64 << 20
    reas = E.DataPlane.Reassembler(uri, E.IPAddress.from_string("::1"), port, 1, rf)
    ok(reas.OpenAndStart())
    ok(seg.OpenAndStart())
    rng = np.random.default_rng(17)
    evs = [rng.integers(0, 256, s, dtype=np.uint8) for s in (1, 1416, 1417, 70000, 1 << 20)]
    for k, e in enumerate(evs):
        ok(seg.addNumpyArrayToSendQueue(e, e.nbytes, 100 + k))
    got = {}
    while len(got) < len(evs):
        n, out, ev, did = reas.recv1DNumpyArray(np.uint8().dtype, 10000)
        assert n > 0, reas.getStats().reassemblyLoss
        got[ev] = out
    seg.stopThreads()
    reas.stopThreads()
    for k, e in enumerate(evs):
        assert np.array_equal(got[100 + k], e)
    assert seg.getSendStats().msgCnt == sum(O.num_packets(e.nbytes, 1416) for e in evs)


# ------------------------------- facade upkeep / reference order -----------------

def _send_raw(port, datagrams):
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 8 << 20)
    for d in datagrams:
        s.sendto(d, (DP, port))
        time.sleep(0)
    s.close()


def _drain_events(reas, n, timeout=20.0):
    got = {}
    deadline = time.time() + timeout
    while len(got) < n and time.time() < deadline:
        r = reas.getEventBytes()
        if r[0] < 0:
            time.sleep(0.002)
            continue
        got[r[2]] = r[1]
    return got


def test_streaming_more_events_than_table_slots(E):
    # 600 five-datagram events through a 64-slot table, each event's tail sent after the
    # next event's head, so an event is always in progress: completed slots must be
    # compacted away while events are in flight (a recycle never gets the chance), with no
    # table exhaustion, no data errors and every event received intact
    port = next_port()
    uri = E.EjfatURI(f"ejfat://useless@192.168.100.1:9875/lb/1?sync=192.168.0.1:12345&data={DP}",
                     E.EjfatURI.TokenType.instance)
    f = E.DataPlane.Reassembler.ReassemblerFlags()
    f.useCP = False
    f.withLBHeader = True
    f.rcvSocketBufSize = 8 << 20
    f.arenaBytes = 64 << 20
    f.tableSlots = 64
    f.recvBatch = 64
    f.recvStride = 128
    f.batchTimeout_us = 100
    reas = E.DataPlane.Reassembler(uri, E.IPAddress.from_string(DP), port, 1, f)
    ok(reas.OpenAndStart())
    mp = O.max_pld_len(80)
    n_ev = 600
    evs, frags = [], []
    for k in range(n_ev):
        ev = np.random.default_rng(9000 + k).integers(0, 256, 67, dtype=np.uint8)
        pk, ln = O.segment_event(ev, 5000 + k, 7, 1, 2, 2, mp)
        evs.append(ev.tobytes())
        frags.append([pk[j, : int(ln[j])].tobytes() for j in range(len(ln))])
    order = list(frags[0][:3])
    for k in range(1, n_ev):
        order += frags[k][:3] + frags[k - 1][3:]
    order += frags[n_ev - 1][3:]
    for i in range(0, len(order), 200):
        _send_raw(port, order[i:i + 200])
        time.sleep(0.005)
    got = _drain_events(reas, n_ev)
    st = reas.getStats()
    ds = reas.getDeviceStats()
    reas.stopThreads()
    assert len(got) == n_ev, (len(got), st.dataErrCnt, ds.errorFlags, ds.tableUsed)
    assert all(got[5000 + k] == evs[k] for k in range(n_ev))
    assert st.dataErrCnt == 0 and st.eventSuccess == n_ev and ds.errorFlags == 0
    assert ds.upkeeps > 0


@pytest.mark.parametrize("reference_order", [False, True])
def test_late_offset0_through_the_facade(E, reference_order):
    # fragments 1, 0, 2, 3, 4 of one event: the reference replaces the item when offset 0
    # arrives late (e2sarDPReassembler.cpp:361-369), so the event never completes and GC
    # logs the new item lost with 4 fragments; the default device path completes it
    port = next_port()
    uri = E.EjfatURI(f"ejfat://useless@192.168.100.1:9875/lb/1?sync=192.168.0.1:12345&data={DP}",
                     E.EjfatURI.TokenType.instance)
    f = E.DataPlane.Reassembler.ReassemblerFlags()
    f.useCP = False
    f.withLBHeader = True
    f.eventTimeout_ms = 200
    f.referenceOrder = reference_order
    f.arenaBytes = 16 << 20
    reas = E.DataPlane.Reassembler(uri, E.IPAddress.from_string(DP), port, 1, f)
    ok(reas.OpenAndStart())
    mp = O.max_pld_len(80)
    pk, ln = O.segment_event(np.frombuffer(SEND_STR, np.uint8), 77, 3, 5, 6, 2, mp)
    for j in (1, 0, 2, 3, 4):
        _send_raw(port, [pk[j, : int(ln[j])].tobytes()])
        time.sleep(0.02)                       # one datagram per batch: arrival order kept
    if reference_order:
        deadline = time.time() + 5
        lost = ()
        while time.time() < deadline and lost == ():
            time.sleep(0.05)
            lost = reas.get_LostEvent()
        assert lost == (77, 3, 4)
        st = reas.getStats()
        assert st.eventSuccess == 0 and st.reassemblyLoss == 1
    else:
        got = _drain_events(reas, 1, timeout=5)
        assert got == {77: SEND_STR}
    reas.stopThreads()


def test_mtu_auto_detect_from_the_outgoing_interface(E):
    # mtu 0: the MTU of the interface the data address routes through
    # (e2sarDPSegmenter.cpp:56-110).  The reference carries it as u_int16_t
    # (e2sarNetUtil.cpp:147-149), so loopback's 65536 reads as 0 and mtu 0 is refused with
    # the reference's message; an override is accepted as is ("lo doesn't" report an MTU)
    port = next_port()
    with pytest.raises(Exception, match="reported as 0"):
        make_seg(E, port, mtu=0)
    seg2 = make_seg(E, port, mtu=1500)
    assert seg2.getIntf() == "lo" and seg2.getMTU() == 1500


# ------------------------------- queue capacities -------------

def test_event_queue_is_unbounded_2000_events_undrained(E):
    """The reference's receive queue is boost::lockfree::queue<EventQueueItem*>{QSIZE} without
    fixed_sized (e2sarDPReassembler.hpp:126-127): QSIZE (1000) pre-sizes its node pool and
    push() allocates beyond it, so a caller that drains late still gets every event and
    enqueueLoss stays 0.  2000 events are sent and reassembled before anything is drained."""
    port = next_port()
    reas = make_reas(E, port)
    ok(reas.OpenAndStart())
    seg = make_seg(E, port, mtu=1500, sockets=1)
    ok(seg.OpenAndStart())
    n = 2000
    rng = np.random.default_rng(20002)
    payloads = [rng.integers(0, 256, 200 + (i * 37) % 3000, dtype=np.uint8).tobytes() for i in range(n)]
    for k, p in enumerate(payloads):
        ok(seg.sendEvent(p, len(p)))
        if k % 200 == 199:
            time.sleep(0.02)                 # keep the loopback socket buffer from overflowing
    deadline = time.time() + 30
    while time.time() < deadline and reas.getStats().eventSuccess < n:
        time.sleep(0.05)
    st = reas.getStats()
    assert st.eventSuccess == n and st.enqueueLoss == 0 and st.reassemblyLoss == 0, \
        (st.eventSuccess, st.enqueueLoss, st.reassemblyLoss)
    got = {}
    for _ in range(n):
        ln, data, ev, did = reas.getEventBytes()
        assert ln >= 0 and did == DATA_ID
        got[ev] = data
    assert reas.getEventBytes()[0] == -1
    assert sorted(got) == list(range(n))
    assert all(got[k] == payloads[k] for k in range(n))
    assert reas.getStats().enqueueLoss == 0 and reas.get_LostEvent() == ()
    seg.stopThreads()
    reas.stopThreads()


def test_send_queue_full_consumes_an_event_number(E):
    """addToSendQueue takes userEventNum++ before the push can fail (e2sarDPSegmenter.cpp:
    937, 939-946): with the queue full (2047 items, hpp:101) the refused default-numbered
    event still uses up its number, so the next accepted event skips it."""
    port = next_port()
    cap = 2047
    t, got = capture(port, cap + 1, timeout=10.0)
    seg = make_seg(E, port, mtu=1500, sockets=1)
    bufs = [bytes([k & 0xFF]) * 64 for k in range(cap + 2)]    # kept alive until sent
    for k in range(cap):                     # not started yet: nothing drains the queue
        ok(seg.addToSendQueue(bufs[k], len(bufs[k])))
    r = seg.addToSendQueue(bufs[cap], len(bufs[cap]))
    assert r.has_error()                     # MemoryError, "Send queue is temporarily full"
    ok(seg.OpenAndStart())
    deadline = time.time() + 20                # let the send thread drain the queue (a retry
    while time.time() < deadline and seg.getSendStats().msgCnt < cap:   # would consume numbers too)
        time.sleep(0.01)
    ok(seg.addToSendQueue(bufs[cap + 1], len(bufs[cap + 1])))
    seg.stopThreads()                        # drains the queue first
    t.join()
    assert len(got) == cap + 1
    evs = {}
    for d in got:
        okv, did, off, blen, ev, _ = O.re_parse(d[16:36])
        assert okv and did == DATA_ID and off == 0 and blen == 64
        evs[ev] = d[36:]
    assert sorted(evs) == list(range(cap)) + [cap + 1]        # number `cap` was consumed
    assert evs[cap + 1] == bufs[cap + 1] and evs[0] == bufs[0] and evs[cap - 1] == bufs[cap - 1]
