"""e2sar_py surface that needs no GPU: header classes, flags, INI, URI, port ranges.
Mirrors test/mem_tests.cpp, test/boost_test.cpp:171-179, DPSegTest5 / DPReasTest5 and
DPReasTest3's get_PortRange table (test/e2sar_reas_test.cpp:345-401)."""
import os

import pytest

import oracle_ffi as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def E():
    from e2sar_amd import e2sar_py
    return e2sar_py


def test_module_constants(E):
    assert E._total_hdr_len == 64 and E._iphdr_len == 20 and E._udphdr_len == 8
    assert E._rehdr_version_nibble == 0x10 and E._dp_port == 19522


def test_rehdr_bytes_match_oracle(E):
    h = E.REHdr()
    h.set(4321, 1436, 1 << 20, 0x0123456789ABCDEF)
    ref = O.lbre_hdr(2, 0, 0, 4321, 1436, 1 << 20, 0x0123456789ABCDEF)[16:]
    assert h.to_bytes() == ref
    assert h.get_fields() == (4321, 1436, 1 << 20, 0x0123456789ABCDEF)
    assert h.validate() and h.get_headerVersion() == 1
    h2 = E.REHdr.from_bytes(ref)
    assert h2.get_eventNum() == 0x0123456789ABCDEF
    assert not E.REHdr.from_bytes(b"\x20" + ref[1:]).validate()


def test_lb_headers_match_oracle(E):
    l2 = E.LBHdrV2()
    l2.set(0xBEEF, 0x0123456789ABCDEF)
    assert l2.to_bytes() == O.lbre_hdr(2, 0xBEEF, 0x0123456789ABCDEF, 0, 0, 0, 0)[:16]
    assert l2.get_fields() == (2, 1, 0xBEEF, 0x0123456789ABCDEF)
    l3 = E.LBHdrV3()
    l3.set(0xCDEF, 0xBEEF, 0x0123456789ABCDEF)   # _send: slot = tick & 0xFFFF
    assert l3.to_bytes() == O.lbre_hdr(3, 0xBEEF, 0x0123456789ABCDEF, 0, 0, 0, 0)[:16]
    # mem_tests.cpp:103-120: lb3.set(1,2,3) decodes as 1 2 3
    l3.set(1, 2, 3)
    assert (l3.get_slotSelect(), l3.get_portSelect(), l3.get_tick()) == (1, 2, 3)
    assert l3.get_version() == 3 and l3.get_nextProto() == 1


def test_sync_header(E):
    s = E.SyncHdr()
    s.set(0x11223344, 77, 1000, 123456789)
    b = s.to_bytes()
    assert len(b) == 28 and b[:4] == b"LC\x02\x00"
    assert s.get_fields() == (0x11223344, 77, 1000, 123456789)


def test_flag_defaults_match_reference(E):
    f = E.DataPlane.Segmenter.SegmenterFlags()       # e2sarDPSegmenter.hpp:384-389
    assert (f.dpV6, f.connectedSocket, f.useCP, f.warmUpMs, f.syncPeriodMs, f.syncPeriods, f.mtu,
            f.numSendSockets, f.sndSocketBufSize, f.rateGbps, f.smooth, f.multiPort, f.ticksAsREEventNum,
            f.lbHdrVersion) == (False, True, True, 1000, 1000, 2, 1500, 4, 3 * 1024 * 1024, -1.0, False, False,
                                False, 2)
    r = E.DataPlane.Reassembler.ReassemblerFlags()   # e2sarDPReassembler.hpp:441-446
    assert (r.useCP, r.useHostAddress, r.period_ms, r.validateCert, r.epoch_ms, r.portRange, r.withLBHeader,
            r.eventTimeout_ms, r.rcvSocketBufSize) == (True, False, 100, True, 1000, -1, False, 500, 3 * 1024 * 1024)


def test_ini_round_trip_like_dpsegtest5(E, tmp_path):
    p = tmp_path / "segmenter.ini"
    p.write_text("[general]\nuseCP = false\n[data-plane]\nsndSocketBufSize = 10000\n")
    res = E.DataPlane.Segmenter.SegmenterFlags.getFromINI(str(p))
    assert not res.has_error()
    f = res.value()
    assert f.useCP is False and f.dpV6 is False and f.sndSocketBufSize == 10000


def test_ini_round_trip_like_dpreastest5(E, tmp_path):
    p = tmp_path / "reassembler.ini"
    p.write_text("[general]\nuseCP = false\n[control-plane]\nuseHostAddress = true\n"
                 "[data-plane]\nrcvSocketBufSize = 10000\n")
    res = E.DataPlane.Reassembler.ReassemblerFlags.getFromINI(str(p))
    f = res.value()
    assert f.useCP is False and f.useHostAddress is True and f.validateCert is True and f.rcvSocketBufSize == 10000


def test_reference_ini_files(E):
    # the reference's own test INI files (test/py_test/*.ini), kept as fixtures
    f = E.DataPlane.Segmenter.SegmenterFlags.getFromINI(os.path.join(GOLDEN, "ref_segmenter_config.ini")).value()
    assert f.mtu == 9000 and f.rateGbps == 10.0 and f.numSendSockets == 4 and f.lbHdrVersion == 2
    assert f.warmUpMs == 1000          # the reference reads this key as bool (cpp:969); fixed here
    r = E.DataPlane.Reassembler.ReassemblerFlags.getFromINI(os.path.join(GOLDEN, "ref_reassembler_config.ini")).value()
    assert r.eventTimeout_ms == 500 and r.portRange == -1 and r.withLBHeader is False
    assert r.Kd == 0.0 and r.weight == 1.0 and r.max_factor == 2.0   # reference overwrites Kd (cpp:714-716)
    missing = E.DataPlane.Segmenter.SegmenterFlags.getFromINI("/nonexistent.ini")
    assert missing.has_error() and missing.error().code == E.E2SARErrorc.ParameterNotAvailable


@pytest.mark.parametrize("n,pr", [(0, 0), (1, 0), (2, 1), (3, 2), (4, 2), (7, 3), (8, 3), (9, 4), (16384, 14),
                                  (20000, 14)])
def test_port_range(E, n, pr):
    # e2sarCP.hpp:772-798; DPReasTest3 uses 1 -> 0, 4 -> 2, 7 -> 3
    assert E._get_PortRange(n) == pr


def test_uri(E):
    u = E.EjfatURI("ejfat://useless@192.168.100.1:9875/lb/1?sync=192.168.0.1:12345&data=127.0.0.1:10000",
                   E.EjfatURI.TokenType.instance)
    assert u.has_data_addr() and u.has_data_addr_v4() and u.has_sync_addr() and not u.has_data_addr_v6()
    assert u.get_lb_id() == "1"
    with pytest.raises(E.E2SARException):
        E.EjfatURI("http://nope")
