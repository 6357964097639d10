"""ctypes access to the CPU oracle (oracle/e2sar_oracle.c) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "build", "libe2sar_oracle.so")


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "enqueueLoss", "reassemblyLoss", "eventSuccess", "totalBytes", "totalPackets",
        "badHeaderDiscards", "dataErrCnt", "inProgress")]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
        L = C.CDLL(ORACLE_LIB)
        vp, sz, u8p = C.c_void_p, C.c_size_t, C.c_void_p
        L.e2o_total_hdr_len.restype = sz
        L.e2o_total_hdr_len.argtypes = [C.c_int]
        L.e2o_max_pld_len.restype = sz
        L.e2o_max_pld_len.argtypes = [C.c_uint, C.c_int]
        L.e2o_num_packets.restype = sz
        L.e2o_num_packets.argtypes = [sz, sz]
        L.e2o_lbre_hdr.restype = None
        L.e2o_lbre_hdr.argtypes = [u8p, C.c_int, C.c_uint16, C.c_uint64, C.c_uint16, C.c_uint32,
                                   C.c_uint32, C.c_uint64]
        L.e2o_re_parse.restype = C.c_int
        L.e2o_re_parse.argtypes = [u8p, C.POINTER(C.c_uint16), C.POINTER(C.c_uint32),
                                   C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_uint8)]
        L.e2o_segment_event.restype = sz
        L.e2o_segment_event.argtypes = [u8p, sz, C.c_uint64, C.c_uint16, C.c_uint16, C.c_uint64,
                                        C.c_int, sz, u8p, sz, u8p]
        L.e2o_reas_new.restype = vp
        L.e2o_reas_new.argtypes = [C.c_int, sz]
        L.e2o_reas_free.restype = None
        L.e2o_reas_free.argtypes = [vp]
        L.e2o_reas_set_time.restype = None
        L.e2o_reas_set_time.argtypes = [vp, C.c_uint64]
        L.e2o_reas_push.restype = None
        L.e2o_reas_push.argtypes = [vp, u8p, sz]
        L.e2o_reas_last_pop_frags.restype = C.c_uint64
        L.e2o_reas_last_pop_frags.argtypes = [vp]
        L.e2o_reas_push_batch.restype = None
        L.e2o_reas_push_batch.argtypes = [vp, u8p, sz, sz, u8p]
        L.e2o_reas_pop.restype = C.c_int
        L.e2o_reas_pop.argtypes = [vp, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(sz), C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_uint16)]
        L.e2o_free.restype = None
        L.e2o_free.argtypes = [vp]
        L.e2o_reas_pop_into.restype = C.c_longlong
        L.e2o_reas_pop_into.argtypes = [vp, u8p, sz, C.POINTER(C.c_uint64), C.POINTER(C.c_uint16)]
        L.e2o_reas_gc.restype = sz
        L.e2o_reas_gc.argtypes = [vp, C.c_uint64]
        L.e2o_reas_lost_pop.restype = C.c_int
        L.e2o_reas_lost_pop.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint16),
                                        C.POINTER(C.c_uint64)]
        L.e2o_reas_get_stats.restype = None
        L.e2o_reas_get_stats.argtypes = [vp, C.POINTER(Stats)]
        L.e2o_cpu_bench.restype = C.c_int
        L.e2o_cpu_bench.argtypes = [u8p, sz, sz, C.c_int, sz, C.c_uint16, C.c_int, C.c_double, sz,
                                    C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def max_pld_len(mtu: int, v6: bool = False) -> int:
    return int(lib().e2o_max_pld_len(mtu, int(v6)))


def num_packets(nbytes: int, max_pld: int) -> int:
    return int(lib().e2o_num_packets(nbytes, max_pld))


def lbre_hdr(ver, entropy, tick, data_id, off, length, event_num) -> bytes:
    out = np.zeros(36, np.uint8)
    lib().e2o_lbre_hdr(_ptr(out), ver, entropy, tick, data_id, off, length, event_num)
    return out.tobytes()


def re_parse(re: bytes):
    a = np.frombuffer(re[:20], np.uint8).copy()
    d, o, l, e, v = C.c_uint16(), C.c_uint32(), C.c_uint32(), C.c_uint64(), C.c_uint8()
    ok = lib().e2o_re_parse(_ptr(a), C.byref(d), C.byref(o), C.byref(l), C.byref(e), C.byref(v))
    return bool(ok), d.value, o.value, l.value, e.value, v.value


def segment_event(event: np.ndarray, event_num: int, data_id: int, entropy: int, tick: int,
                  ver: int, max_pld: int, stride: int | None = None):
    """-> (packets[n, stride] uint8, lens[n] uint32)"""
    event = np.ascontiguousarray(event, dtype=np.uint8)
    n = num_packets(event.size, max_pld)
    stride = stride or (36 + max_pld)
    pk = np.zeros((max(n, 1), stride), np.uint8)
    ln = np.zeros(max(n, 1), np.uint32)
    got = lib().e2o_segment_event(_ptr(event) if event.size else None, event.size, event_num, data_id,
                                  entropy, tick, ver, max_pld, _ptr(pk), stride, _ptr(ln))
    assert got == n
    return pk[:n], ln[:n]


class Reassembler:
    """The reference recv body restated (e2sarDPReassembler.cpp:310-428)."""

    def __init__(self, with_lb_header: bool, queue_capacity: int = 0):
        """queue_capacity 0: the reference's unbounded eventQueue (hpp:126-127); nonzero: a
        device completed-record ring of that capacity (not reference behaviour)"""
        self.h = lib().e2o_reas_new(int(with_lb_header), queue_capacity)

    def set_time(self, ms: int):
        lib().e2o_reas_set_time(self.h, ms)

    def push(self, dgram: bytes | np.ndarray):
        a = np.frombuffer(bytes(dgram), np.uint8).copy() if not isinstance(dgram, np.ndarray) else dgram
        lib().e2o_reas_push(self.h, _ptr(a) if a.size else None, a.size)

    def push_batch(self, pkts: np.ndarray, lens: np.ndarray):
        pkts = np.ascontiguousarray(pkts, np.uint8)
        lens = np.ascontiguousarray(lens, np.uint32)
        lib().e2o_reas_push_batch(self.h, _ptr(pkts), len(lens), pkts.shape[1], _ptr(lens))

    def pop(self, cap: int = 1 << 26):
        buf = np.empty(cap, np.uint8)
        ev, d = C.c_uint64(), C.c_uint16()
        n = lib().e2o_reas_pop_into(self.h, _ptr(buf), cap, C.byref(ev), C.byref(d))
        if n == -1:
            return None
        if n == -2:
            raise ValueError("event larger than pop buffer")
        return buf[:n].tobytes(), ev.value, d.value

    def pop_all_frags(self, cap: int = 1 << 26):
        """(bytes, eventNum, dataId, numFragments) of every queued event."""
        out = []
        while True:
            r = self.pop(cap)
            if r is None:
                return out
            out.append(r + (int(lib().e2o_reas_last_pop_frags(self.h)),))

    def pop_all(self, cap: int = 1 << 26):
        out = []
        while True:
            r = self.pop(cap)
            if r is None:
                return out
            out.append(r)

    def gc(self, timeout_ms: int) -> int:
        return int(lib().e2o_reas_gc(self.h, timeout_ms))

    def lost_pop_all(self):
        out = []
        ev, d, nf = C.c_uint64(), C.c_uint16(), C.c_uint64()
        while lib().e2o_reas_lost_pop(self.h, C.byref(ev), C.byref(d), C.byref(nf)) == 0:
            out.append((ev.value, d.value, nf.value))
        return out

    def stats(self) -> dict:
        s = Stats()
        lib().e2o_reas_get_stats(self.h, C.byref(s))
        return {n: getattr(s, n) for n, _ in Stats._fields_}

    def __del__(self):
        try:
            lib().e2o_reas_free(self.h)
        except Exception:
            pass
