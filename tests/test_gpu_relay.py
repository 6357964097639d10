"""BASELINE config 5's on-device relay chain against the oracle.

reassemble_batch (the receive body, e2sarDPReassembler.cpp:335-427) -> relay_plan_kernel
(completed records -> seg descriptors, no host round trip) -> segment_batch_dev (the
_send fragment loop, e2sarDPSegmenter.cpp:702-770, with the event count read on the
device).  Every re-sent datagram's bytes and length must equal the oracle's segmentation
of the reassembled event with the relay's per-event rules (include/e2sar_hip.h: RE
eventNum and dataId as received, one LB tick for the batch, entropy of the i-th planned
event = entropyBase + i mod 2^16).
"""
import numpy as np
import pytest

import oracle_ffi as O

pytestmark = pytest.mark.gpu

SEG_EVENT = np.dtype([("data", "<u8"), ("eventNum", "<u8"), ("lbTick", "<u8"), ("bytes", "<u4"),
                      ("pktBase", "<u4"), ("dataId", "<u2"), ("entropy", "<u2"), ("reserved", "<u4")])
assert SEG_EVENT.itemsize == 40

# ragged: sub-dword, one byte either side of a payload, many datagrams, non-multiples of 4
SIZES = [1, 3, 67, 1435, 1436, 1437, 5000, 8935, 8937, 100001, 1 << 20, (2 << 20) + 7]


def _inputs(seed):
    rnd = np.random.default_rng(seed)
    evs = []
    for k, b in enumerate(SIZES):
        evs.append((rnd.integers(0, 256, b, dtype=np.uint8), 1000 + 3 * k, 4321 + (k % 3)))
    return evs


@pytest.mark.parametrize("mtu_in,mtu_out,ver", [(1500, 1500, 2), (1500, 1500, 3), (9000, 9000, 2),
                                                (9000, 9000, 3), (9000, 1500, 2), (1500, 1499, 3)])
def test_relay_chain_matches_the_oracle(hip, mtu_in, mtu_out, ver):
    import torch
    from e2sar_amd import sar
    evs = _inputs(mtu_in + 7 * mtu_out + ver)
    # the datagrams the relay receives: the oracle's segmentation, in order, LB header kept
    mp_in = O.max_pld_len(mtu_in)
    stride_in = sar.packet_stride(mp_in)
    pks, lns = [], []
    for k, (b, e, d) in enumerate(evs):
        p, l = O.segment_event(b, e, d, 0x100 + k, 0xABC00 + k, 2, mp_in, stride_in)
        pks.append(p)
        lns.append(l)
    pk = np.concatenate(pks)
    ln = np.concatenate(lns).astype(np.uint32)
    n_in = len(ln)
    dpk = torch.from_numpy(pk.reshape(-1)).to(hip.torch_device)
    dln = torch.from_numpy(ln.view(np.int32)).to(hip.torch_device)
    R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=256, queue_capacity=256, lost_capacity=64,
                              arena_bytes=64 << 20)
    seg = sar.DeviceSegmenter(hip, mtu=mtu_out, lb_hdr_version=ver)
    nev = len(evs)
    maxpk = max((len(b) + seg.max_pld - 1) // seg.max_pld for b, _, _ in evs)
    desc = torch.zeros(nev * sar.SEG_EVENT_BYTES, dtype=torch.uint8, device=hip.torch_device)
    cnt = torch.zeros(2, dtype=torch.int32, device=hip.torch_device)
    opk, oln = seg.alloc_packets(nev * maxpk)
    tick, ent0 = 0x0123456789ABCDEF, 0xFFFD               # entropies wrap past 0xFFFF
    R.reassemble(dpk, stride_in, dln, n_in)
    R.relay_plan(desc, cnt, 0, nev, seg.max_pld, tick, ent0)
    seg.segment_device(desc, cnt, nev, maxpk, opk, oln)
    torch.cuda.synchronize()
    n, total = (int(x) for x in cnt.cpu().tolist())
    recs = R.poll()
    assert n == nev == len(recs)
    assert R.stats().eventSuccess == nev
    table = np.frombuffer(desc.cpu().numpy().tobytes(), SEG_EVENT)[:n]
    by_key = {(e, d): b for b, e, d in evs}
    gp = opk[: total * seg.stride].view(total, seg.stride).cpu().numpy()
    gl = oln[:total].cpu().numpy().astype(np.uint32)
    base = 0
    for i, (t, rec) in enumerate(zip(table, recs)):
        # descriptor i is completed record i: its arena bytes, key, the batch's tick and entropy
        assert int(t["data"]) == R.arena_ptr + rec.arenaOffset
        assert (int(t["eventNum"]), int(t["dataId"])) == (rec.eventNum, rec.dataId)
        assert int(t["lbTick"]) == tick and int(t["entropy"]) == (ent0 + i) & 0xFFFF
        assert int(t["bytes"]) == rec.bytes and int(t["pktBase"]) == base
        b = by_key[(rec.eventNum, rec.dataId)]
        op, ol = O.segment_event(b, rec.eventNum, rec.dataId, (ent0 + i) & 0xFFFF, tick, ver, seg.max_pld, seg.stride)
        np_ = len(ol)
        np.testing.assert_array_equal(gl[base:base + np_], ol)
        for k in range(np_):
            L = int(ol[k])
            assert np.array_equal(gp[base + k, :L], op[k, :L]), (i, k, L)
        base += np_
    assert base == total
    R.close()


def _relay_and_check(hip, evs, mtu_in, mtu_out, ver, tick, ent0):
    """One relay pass over events evs [(bytes, eventNum, dataId)] against the oracle."""
    import torch
    from e2sar_amd import sar
    mp_in = O.max_pld_len(mtu_in)
    stride_in = sar.packet_stride(mp_in)
    pks, lns = [], []
    for k, (b, e, d) in enumerate(evs):
        p, l = O.segment_event(b, e, d, 0x100 + k, 0xABC00 + k, 2, mp_in, stride_in)
        pks.append(p)
        lns.append(l)
    pk = np.concatenate(pks)
    ln = np.concatenate(lns).astype(np.uint32)
    dpk = torch.from_numpy(pk.reshape(-1)).to(hip.torch_device)
    dln = torch.from_numpy(ln.view(np.int32)).to(hip.torch_device)
    total_bytes = sum(len(b) for b, _, _ in evs)
    R = sar.DeviceReassembler(hip, with_lb_header=True, table_slots=256, queue_capacity=256, lost_capacity=64,
                              arena_bytes=total_bytes + 256 * (len(evs) + 1))
    seg = sar.DeviceSegmenter(hip, mtu=mtu_out, lb_hdr_version=ver)
    nev = len(evs)
    maxpk = max((len(b) + seg.max_pld - 1) // seg.max_pld for b, _, _ in evs)
    desc = torch.zeros(nev * sar.SEG_EVENT_BYTES, dtype=torch.uint8, device=hip.torch_device)
    cnt = torch.zeros(2, dtype=torch.int32, device=hip.torch_device)
    opk, oln = seg.alloc_packets(nev * maxpk)
    R.reassemble(dpk, stride_in, dln, len(ln))
    R.relay_plan(desc, cnt, 0, nev, seg.max_pld, tick, ent0)
    seg.segment_device(desc, cnt, nev, maxpk, opk, oln)
    torch.cuda.synchronize()
    n, total = (int(x) for x in cnt.cpu().tolist())
    recs = R.poll()
    assert n == nev == len(recs)
    by_key = {(e, d): b for b, e, d in evs}
    gp = opk[: total * seg.stride].view(total, seg.stride).cpu().numpy()
    gl = oln[:total].cpu().numpy().astype(np.uint32)
    base = 0
    for i, rec in enumerate(recs):
        b = by_key[(rec.eventNum, rec.dataId)]
        op, ol = O.segment_event(b, rec.eventNum, rec.dataId, (ent0 + i) & 0xFFFF, tick, ver, seg.max_pld, seg.stride)
        np.testing.assert_array_equal(gl[base:base + len(ol)], ol)
        for k in range(len(ol)):
            L = int(ol[k])
            assert np.array_equal(gp[base + k, :L], op[k, :L]), (i, k, L)
        base += len(ol)
    assert base == total
    R.close()


@pytest.mark.parametrize("seed", range(12))
def test_relay_chain_random(hip, seed):
    """Random batches: event count, sizes (1 B up, not dword multiples), MTU in and out
    (80 .. 9000), LB version, tick and entropy base, all drawn from the seed."""
    rnd = np.random.default_rng(0x5E1A + seed)
    mtus = [80, 577, 1500, 4000, 9000]
    mtu_in = int(rnd.choice(mtus))
    mtu_out = int(rnd.choice(mtus))
    ver = int(rnd.choice([2, 3]))
    # at most ~60 K datagrams either side
    cap = 60_000 * min(O.max_pld_len(mtu_in), O.max_pld_len(mtu_out))
    nev = int(rnd.integers(1, 40))
    sizes = [int(x) for x in rnd.integers(1, max(2, min(400_000, cap // nev)), nev)]
    evs = [(rnd.integers(0, 256, s, dtype=np.uint8), int(rnd.integers(0, 1 << 62)), int(rnd.integers(0, 1 << 16)))
           for s in sizes]
    keys = {(e, d) for _, e, d in evs}
    assert len(keys) == len(evs)
    _relay_and_check(hip, evs, mtu_in, mtu_out, ver, int(rnd.integers(0, 1 << 63)), int(rnd.integers(0, 1 << 16)))
