"""ctypes binding of the C ABI in ``include/e2sar_hip.h``.

The shared library ``e2sar_amd/lib/libe2sar_hip.so`` is built in-tree by
``make`` (or ``__graft_entry__.build()``).  Loading fails loudly when it is
missing: there is no CPU fallback for the SAR path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("E2SAR_HIP_LIB") or os.path.join(_HERE, "lib", "libe2sar_hip.so")

# status codes = -(E2SARErrorc) (reference include/e2sarError.hpp:23-39)
OK = 0
ERR_PARAMETER = -3
ERR_OUT_OF_RANGE = -5
ERR_NOT_FOUND = -7
ERR_MEMORY = -10
ERR_LOGIC = -11
ERR_SYSTEM = -12
ERR_DATA = -13

LBRE_HDR_LEN = 36
RE_HDR_LEN = 20
LB_HDR_LEN = 16


class SegEvent(C.Structure):
    _fields_ = [
        ("data", C.c_uint64),
        ("eventNum", C.c_uint64),
        ("lbTick", C.c_uint64),
        ("bytes", C.c_uint32),
        ("pktBase", C.c_uint32),
        ("dataId", C.c_uint16),
        ("entropy", C.c_uint16),
        ("reserved", C.c_uint32),
    ]


class CopySpan(C.Structure):
    _fields_ = [
        ("src", C.c_uint64),
        ("dst", C.c_uint64),
        ("bytes", C.c_uint64),
    ]


class SegReasBatch(C.Structure):
    _fields_ = [
        ("d_events", C.c_uint64),
        ("d_packets", C.c_uint64),
        ("d_lens", C.c_uint64),
        ("nEvents", C.c_uint32),
        ("maxPacketsPerEvent", C.c_uint32),
        ("nPackets", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class ReasConfig(C.Structure):
    _fields_ = [
        ("withLBHeader", C.c_int),
        ("tableSlots", C.c_uint32),
        ("queueCapacity", C.c_uint32),
        ("lostCapacity", C.c_uint32),
        ("arenaBytes", C.c_uint64),
        ("flags", C.c_uint32),
        ("groupSize", C.c_uint32),
    ]


REAS_COMPACTABLE = 1
REAS_REFERENCE_ORDER = 2      # arrival-order rules of the reference receive body (e2sar_hip.h)
REAS_COLD_DATAGRAMS = 4       # datagrams written long before: streaming loads in the scatter (e2sar_hip.h)


class EventRec(C.Structure):
    _fields_ = [
        ("eventNum", C.c_uint64),
        ("arenaOffset", C.c_uint64),
        ("bytes", C.c_uint32),
        ("dataId", C.c_uint16),
        ("flags", C.c_uint16),
        ("numFragments", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class LostRec(C.Structure):
    _fields_ = [
        ("eventNum", C.c_uint64),
        ("numFragments", C.c_uint64),
        ("dataId", C.c_uint16),
        ("enqueueLoss", C.c_uint16),
        ("reserved", C.c_uint32),
    ]


class ReasStats(C.Structure):
    _fields_ = [
        ("enqueueLoss", C.c_uint64),
        ("reassemblyLoss", C.c_uint64),
        ("eventSuccess", C.c_uint64),
        ("totalPackets", C.c_uint64),
        ("totalBytes", C.c_uint64),
        ("badHeaderDiscards", C.c_uint64),
        ("dataErrCnt", C.c_uint64),
        ("inProgress", C.c_int64),
        ("completedPending", C.c_uint64),
        ("lostPending", C.c_uint64),
        ("arenaUsed", C.c_uint64),
        ("tableUsed", C.c_uint64),
        ("errorFlags", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


assert C.sizeof(SegEvent) == 40
assert C.sizeof(EventRec) == 32
assert C.sizeof(LostRec) == 24

vp = C.c_void_p
u8p = C.c_void_p
i = C.c_int
u32 = C.c_uint32
u64 = C.c_uint64
sz = C.c_size_t

# name -> (restype, argtypes); this list is also the export contract checked by tests
SIGNATURES = {
    "e2sar_hip_abi_version": (i, []),
    "e2sar_hip_last_error": (C.c_char_p, []),
    "e2sar_hip_ctx_create": (i, [i, vp, C.POINTER(vp)]),
    "e2sar_hip_ctx_destroy": (None, [vp]),
    "e2sar_hip_stream_create": (i, [i, C.POINTER(vp)]),
    "e2sar_hip_stream_destroy": (i, [vp]),
    "e2sar_hip_ctx_stream": (vp, [vp]),
    "e2sar_hip_ctx_device": (i, [vp]),
    "e2sar_hip_ctx_sync": (i, [vp]),
    "e2sar_hip_device_alloc": (i, [vp, sz, C.POINTER(vp)]),
    "e2sar_hip_device_free": (i, [vp, vp]),
    "e2sar_hip_host_alloc": (i, [sz, C.POINTER(vp)]),
    "e2sar_hip_host_free": (i, [vp]),
    "e2sar_hip_memcpy_h2d": (i, [vp, vp, vp, sz]),
    "e2sar_hip_memcpy_d2h": (i, [vp, vp, vp, sz]),
    "e2sar_hip_memset_d": (i, [vp, vp, i, sz]),
    "e2sar_hip_memset_async": (i, [vp, vp, i, sz, vp]),
    "e2sar_hip_memcpy_async": (i, [vp, vp, vp, sz, i, vp]),
    "e2sar_hip_stream_sync": (i, [vp, vp]),
    "e2sar_hip_event_create": (i, [vp, C.POINTER(vp)]),
    "e2sar_hip_event_destroy": (i, [vp]),
    "e2sar_hip_event_record": (i, [vp, vp, vp]),
    "e2sar_hip_stream_wait_event": (i, [vp, vp, vp]),
    "e2sar_hip_event_query": (i, [vp]),
    "e2sar_hip_event_sync": (i, [vp]),
    "e2sar_hip_copy_spans": (i, [vp, vp, u32, vp]),
    "e2sar_hip_total_hdr_len": (sz, [i]),
    "e2sar_hip_max_pld_len": (sz, [u32, i]),
    "e2sar_hip_num_packets": (sz, [sz, sz]),
    "e2sar_hip_packet_stride": (u32, [sz]),
    "e2sar_hip_seg_plan": (i, [C.POINTER(SegEvent), u32, sz, C.POINTER(u32), C.POINTER(u32)]),
    "e2sar_hip_segment_batch": (i, [vp, vp, u32, u32, i, u32, i, vp, u32, vp, vp]),
    "e2sar_hip_segment_batch_dev": (i, [vp, vp, vp, u32, u32, i, u32, vp, u32, vp, vp]),
    "e2sar_hip_segment_batch_recycle": (i, [vp, vp, u32, u32, i, u32, i, vp, u32, vp, vp, i, vp]),
    "e2sar_hip_relay_plan": (i, [vp, u32, u32, sz, u64, C.c_uint16, vp, vp, vp]),
    "e2sar_hip_reas_create": (i, [vp, C.POINTER(ReasConfig), C.POINTER(vp)]),
    "e2sar_hip_reas_destroy": (None, [vp]),
    "e2sar_hip_reas_arena": (vp, [vp]),
    "e2sar_hip_reassemble_batch": (i, [vp, vp, u32, vp, u32, u64, vp]),
    "e2sar_hip_reas_work_bytes": (sz, [u32]),
    "e2sar_hip_reas_classify": (i, [vp, vp, u32, vp, u32, u64, vp, sz, vp]),
    "e2sar_hip_reas_scatter": (i, [vp, vp, u32, u32, vp, sz, vp]),
    "e2sar_hip_reas_scatter_classify": (i, [vp, u32, vp, u32, vp, sz, vp, vp, u32, u64, vp, sz, vp]),
    "e2sar_hip_reas_gc": (i, [vp, u64, u64, vp]),
    "e2sar_hip_reas_poll": (i, [vp, C.POINTER(EventRec), u32, C.POINTER(u32)]),
    "e2sar_hip_reas_lost_poll": (i, [vp, C.POINTER(LostRec), u32, C.POINTER(u32)]),
    "e2sar_hip_reas_get_stats": (i, [vp, C.POINTER(ReasStats)]),
    "e2sar_hip_reas_recycle": (i, [vp, i, vp]),
    "e2sar_hip_reas_reset_stats": (i, [vp, vp]),
    "e2sar_hip_reas_compact": (i, [vp, vp]),
    "e2sar_hip_route_workspace_bytes": (sz, [u32, u32]),
    "e2sar_hip_route_batch": (i, [vp, vp, u32, vp, u32, i, u32, u32, vp, vp, vp, vp, sz, vp]),
    "e2sar_hip_route_foreign": (i, [vp, vp, u32, vp, u32, i, u32, u32, vp, vp, vp, vp, sz, vp]),
    "e2sar_hip_route_append": (i, [vp, vp, u32, vp, u32, i, u32, u32, i, vp, vp, u32, vp, vp, sz, vp]),
    "e2sar_hip_reas_set_owner": (i, [vp, u32, u32]),
    "e2sar_hip_reas_set_cold": (i, [vp, i]),
    "e2sar_hip_reas_forget_stream": (i, [vp, vp]),
}

# include/e2sar_hip_experimental.h: A/B-only launch forms, bound when the loaded library
# was built with them (`make experimental`, E2SAR_HIP_LIB=build/variants/lib_experimental.so)
EXPERIMENTAL_SIGNATURES = {
    "e2sar_hip_segment_reassemble_batch": (i, [vp, vp, u32, u32, u32, i, u32, vp, u32, vp, vp, u64, vp]),
    "e2sar_hip_segment_reassemble_batches": (i, [vp, vp, u32, i, u32, u32, vp, u64, vp]),
    "e2sar_hip_seg_groups": (i, [C.POINTER(SegEvent), u32, u32, u32, u32, C.POINTER(u32), u32, C.POINTER(u32)]),
    "e2sar_hip_reassemble_groups": (i, [vp, vp, u32, vp, u32, vp, u32, u64, vp]),
}


class E2SARHipError(RuntimeError):
    """A failing C-ABI call: ``code`` is -(E2SARErrorc)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"E2SAR HIP error {code}: {msg}")
        self.code = code
        self.msg = msg


_lib = None


def lib() -> C.CDLL:
    """Load (once) and return the HIP SAR library; raises if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build()). "
                "The E2SAR SAR path has no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        for name, (res, args) in EXPERIMENTAL_SIGNATURES.items():
            if hasattr(L, name):
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
        _lib = L
    return _lib


def has_experimental() -> bool:
    """True when the library carries the A/B-only forms of e2sar_hip_experimental.h.

    Reads the library's dynamic symbol table without loading it: in a process that also
    uses PyTorch, the library must be loaded only after torch has initialised the GPU (its
    HIP runtime and torch's share one HSA runtime, the first one loaded; sar.Context loads
    the library after torch.cuda.set_device).  Loaded first, this library's runtime finds no
    device.  So a test module's skip marker, evaluated at collection, must not load it."""
    if _lib is not None:
        return all(hasattr(_lib, n) for n in EXPERIMENTAL_SIGNATURES)
    if not os.path.exists(LIB_PATH):
        return False
    return set(EXPERIMENTAL_SIGNATURES) <= elf_defined_symbols(LIB_PATH)


def elf_defined_symbols(path: str) -> set:
    """Names of the symbols an ELF64 little-endian shared library defines (its .dynsym
    entries with a section index), read from the file -- no loader, no binutils."""
    import struct
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
        raise ValueError(f"{path}: not an ELF64 little-endian file")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", data, 0x3A)
    sections = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + k * shentsize) for k in range(shnum)]
    out = set()
    for name, typ, _fl, _addr, off, size, link, _info, _al, entsize in sections:
        if typ != 11 or not entsize:                            # SHT_DYNSYM
            continue
        stroff = sections[link][4]
        for k in range(size // entsize):
            st_name, _st_info, _st_other, st_shndx = struct.unpack_from("<IBBH", data, off + k * entsize)
            if st_shndx == 0 or st_name == 0:                   # undefined / unnamed
                continue
            end = data.index(b"\0", stroff + st_name)
            out.add(data[stroff + st_name:end].decode())
    return out


def need_experimental(what: str) -> None:
    if not has_experimental():
        raise E2SARHipError(ERR_LOGIC, f"{what} is an A/B-only form (include/e2sar_hip_experimental.h): build it "
                                       "with `make experimental` and load E2SAR_HIP_LIB=build/variants/"
                                       "lib_experimental.so")


def check(rc: int) -> int:
    if rc < 0:
        raise E2SARHipError(rc, lib().e2sar_hip_last_error().decode(errors="replace"))
    return rc
