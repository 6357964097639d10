"""Header byte positions pinned by a second definition inside the reference.

`e2sarHeaders.hpp` defines the LB/RE/Sync headers as C++ structs; the reference's packet
sniffer/generator `scripts/scapy/snifgen.py` defines the same wire formats independently,
as scapy field lists (network byte order):

* LBPacket (snifgen.py:38-48): preamble 'LB' (2), version (1) = 2, nextProto (1) = 1,
  rsvd (2), entropy (2), eventNumber (8)                              -> 16 bytes
* REPacket (snifgen.py:67-79): version (4 bits) = 1, rsvd (4 bits), rsvd2 (1), dataId (2),
  bufferOffset (4), bufferLength (4, "Event Length"), eventNumber (8) -> 20 bytes
* SyncPacket (snifgen.py:24-35): preamble 'LC' (2), version (1) = 2, reserved (1),
  eventSrcId (4), eventNumber (8), avgEventRateHz (4), unixTimeNano (8) -> 28 bytes

and its generator genLBREPkt (snifgen.py:107-126) fills bufferOffset with the running
segment offset and bufferLength with the whole payload length.  The struct formats below
restate those field lists; decoding the oracle's datagrams and the committed golden headers
(which the HIP path must reproduce, tests/test_gpu_golden.py) with them pins every field's
byte position to the reference's own second definition, so an oracle that swapped two
fields on both its write and read side would fail here.  The v3 LB header (slotSelect /
portSelect) has no snifgen counterpart; it stays pinned by SURVEY 8(a)'s hex KAT.
"""
import json
import os
import struct

import numpy as np
import pytest

import oracle_ffi as O

HERE = os.path.dirname(os.path.abspath(__file__))
LB_FMT = "!2sBBHHQ"        # snifgen.py:41-46
RE_FMT = "!BBHIIQ"         # snifgen.py:70-76 (version and rsvd share the first byte)
SYNC_FMT = "!2sBBIQIQ"     # snifgen.py:27-33
assert struct.calcsize(LB_FMT) == 16 and struct.calcsize(RE_FMT) == 20 and struct.calcsize(SYNC_FMT) == 28


def decode(hdr: bytes):
    pre, ver, proto, rsvd, entropy, lbev = struct.unpack(LB_FMT, hdr[:16])
    b0, rsvd2, data_id, off, blen, ev = struct.unpack(RE_FMT, hdr[16:36])
    return dict(pre=pre, lbver=ver, proto=proto, rsvd=rsvd, entropy=entropy, lbev=lbev,
                rever=b0 >> 4, rersvd=b0 & 15, rsvd2=rsvd2, dataId=data_id, off=off, blen=blen, ev=ev)


@pytest.mark.parametrize("mtu,size", [(1500, 100000), (9000, 70001), (80, 67), (1500, 1)])
def test_oracle_datagrams_decode_with_the_snifgen_layout(mtu, size):
    mp = O.max_pld_len(mtu)
    stride = (36 + mp + 15) // 16 * 16
    ev = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8)
    event_num, data_id, entropy, tick = 0x0102030405060708, 0x10E1, 0xBEEF, 0x1122334455667788
    pk, ln = O.segment_event(ev, event_num, data_id, entropy, tick, 2, mp, stride)
    assert len(ln) == -(-size // mp)
    for k in range(len(ln)):
        h = decode(pk[k, :36].tobytes())
        assert (h["pre"], h["lbver"], h["proto"], h["rsvd"]) == (b"LB", 2, 1, 0)
        assert h["entropy"] == entropy and h["lbev"] == tick
        assert (h["rever"], h["rersvd"], h["rsvd2"]) == (1, 0, 0)
        # genLBREPkt: running segment offset, whole payload length (snifgen.py:118-121)
        assert h["dataId"] == data_id and h["off"] == k * mp and h["blen"] == size and h["ev"] == event_num
        assert int(ln[k]) == 36 + min(mp, size - k * mp)
        assert pk[k, 36:ln[k]].tobytes() == ev[k * mp: k * mp + ln[k] - 36].tobytes()


def test_golden_headers_decode_with_the_snifgen_layout():
    with open(os.path.join(HERE, "golden", "sar_golden.json")) as f:
        golden = json.load(f)
    n = 0
    for case in golden["segment"]:
        mp, size = case["maxPldLen"], case["bytes"]
        for e in case["events"]:
            for key, k in (("first_hdr", 0), ("second_hdr", 1), ("last_hdr", e["numPackets"] - 1)):
                h = decode(bytes.fromhex(e[key]))
                assert h["pre"] == b"LB" and h["lbver"] == case["lbHdrVersion"] and h["proto"] == 1
                if case["lbHdrVersion"] == 2:       # snifgen defines v2 only
                    assert h["rsvd"] == 0 and h["entropy"] == e["entropy"] and h["lbev"] == e["lbTick"]
                assert (h["rever"], h["rersvd"], h["rsvd2"]) == (1, 0, 0)
                assert h["dataId"] == e["dataId"] and h["off"] == k * mp and h["blen"] == size
                assert h["ev"] == e["eventNum"]
                n += 1
            assert e["last_len"] == 36 + size - (e["numPackets"] - 1) * mp
    assert n == 3 * sum(len(c["events"]) for c in golden["segment"])


def test_header_classes_match_snifgen():
    # the façade's header classes (e2sarHeaders.hpp:21-208, 323-403) through e2sar_py
    from e2sar_amd import e2sar_py
    sync = e2sar_py.SyncHdr()
    sync.set(0x01020304, 0x1122334455667788, 0x0A0B0C0D, 0x99AABBCCDDEEFF00)
    pre, ver, rsvd, src, ev, rate, ns = struct.unpack(SYNC_FMT, sync.to_bytes())
    assert (pre, ver, rsvd) == (b"LC", 2, 0)
    assert (src, ev, rate, ns) == (0x01020304, 0x1122334455667788, 0x0A0B0C0D, 0x99AABBCCDDEEFF00)
    lb = e2sar_py.LBHdrV2()
    lb.set(0xBEEF, 0x0123456789ABCDEF)
    assert struct.unpack(LB_FMT, lb.to_bytes()) == (b"LB", 2, 1, 0, 0xBEEF, 0x0123456789ABCDEF)
    re = e2sar_py.REHdr()
    re.set(0x10E1, 1436, 1 << 20, 0x0102030405060708)
    assert struct.unpack(RE_FMT, re.to_bytes()) == (0x10, 0, 0x10E1, 1436, 1 << 20, 0x0102030405060708)


# LBHdrV3 as e2sarHeaders.hpp:191-198 declares it (packed, network byte order): preamble
# char[2] 'LB', version u8 (lbhdrVersion3 = 3), nextProto u8 (rehdrVersion = 1),
# slotSelect u16, portSelect u16, tick u64 -- and _send fills it with
# lb3.set(lbEventNum & 0xFFFF, entropy, lbEventNum) (e2sarDPSegmenter.cpp:753).  This is a
# restatement of the reference's own struct, not a second independent definition (snifgen
# has none for v3), so it pins the member order the header declares; DESIGN.md 5.1 records
# that no reference-held vector covers v3 bytes.
LB3_FMT = "!2sBBHHQ"        # e2sarHeaders.hpp:193-198
assert struct.calcsize(LB3_FMT) == 16


def decode_v3(hdr: bytes):
    pre, ver, proto, slot, port, tick = struct.unpack(LB3_FMT, hdr[:16])
    return dict(pre=pre, ver=ver, proto=proto, slot=slot, port=port, tick=tick)


def test_v3_headers_decode_with_the_reference_struct_order():
    mp = O.max_pld_len(1500)
    stride = (36 + mp + 15) // 16 * 16
    ev = np.random.default_rng(3).integers(0, 256, 5000, dtype=np.uint8)
    entropy, tick = 0xBEEF, 0x0123456789ABCDEF
    pk, ln = O.segment_event(ev, 7, 0x10E1, entropy, tick, 3, mp, stride)
    for k in range(len(ln)):
        h = decode_v3(pk[k, :16].tobytes())
        assert (h["pre"], h["ver"], h["proto"]) == (b"LB", 3, 1)
        assert h["slot"] == tick & 0xFFFF and h["port"] == entropy and h["tick"] == tick
    with open(os.path.join(HERE, "golden", "sar_golden.json")) as f:
        golden = json.load(f)
    n = 0
    for case in golden["segment"]:
        if case["lbHdrVersion"] != 3:
            continue
        for e in case["events"]:
            for key in ("first_hdr", "second_hdr", "last_hdr"):
                h = decode_v3(bytes.fromhex(e[key]))
                assert (h["pre"], h["ver"], h["proto"]) == (b"LB", 3, 1)
                assert h["slot"] == e["lbTick"] & 0xFFFF and h["port"] == e["entropy"] and h["tick"] == e["lbTick"]
                n += 1
    assert n > 0
