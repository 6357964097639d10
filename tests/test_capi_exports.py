"""The C-ABI library loads and exports every symbol include/e2sar_hip.h declares
(CPU only: no compute calls), and the host-only geometry entry points agree with the
oracle."""
import os
import re
import subprocess

import pytest

import oracle_ffi as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "e2sar_hip.h")


def declared_functions(header=HEADER):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(e2sar_hip_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    for must in ("e2sar_hip_segment_batch", "e2sar_hip_reassemble_batch", "e2sar_hip_reas_poll",
                 "e2sar_hip_max_pld_len", "e2sar_hip_ctx_create"):
        assert must in fns


def test_library_exports_every_declared_symbol():
    from e2sar_amd import _capi
    L = _capi.lib()
    for fn in declared_functions():
        assert hasattr(L, fn), fn
    assert set(declared_functions()) == set(_capi.SIGNATURES), "ctypes table out of sync with header"
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (e2sar_hip_\w+)", out))
    assert set(declared_functions()) <= exported


def test_experimental_forms_are_not_in_the_product():
    # the A/B-only launch forms (no gain on any BASELINE config) live in
    # e2sar_hip_experimental.h and build/variants/lib_experimental.so only
    from e2sar_amd import _capi
    exp = declared_functions(os.path.join(ROOT, "include", "e2sar_hip_experimental.h"))
    assert set(exp) == set(_capi.EXPERIMENTAL_SIGNATURES)
    assert not set(exp) & set(declared_functions())
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (e2sar_hip_\w+)", out))
    if _capi.LIB_PATH.endswith("lib/libe2sar_hip.so"):
        assert not set(exp) & exported


def test_elf_symbol_reader_matches_nm():
    """has_experimental() reads the library's .dynsym in Python (no binutils on the path, no
    load before torch); it must see what nm sees, and tell the product library from the
    experimental one."""
    import shutil
    from e2sar_amd import _capi
    mine = {n for n in _capi.elf_defined_symbols(_capi.LIB_PATH) if n.startswith("e2sar_hip_")}
    assert set(declared_functions()) <= mine
    if shutil.which("nm"):
        out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True).stdout
        assert mine == set(re.findall(r" [TW] (e2sar_hip_\w+)", out))
    if _capi.LIB_PATH.endswith("lib/libe2sar_hip.so"):
        assert not _capi.has_experimental()
    exp_lib = os.path.join(ROOT, "build", "variants", "lib_experimental.so")
    if os.path.exists(exp_lib):
        assert set(_capi.EXPERIMENTAL_SIGNATURES) <= _capi.elf_defined_symbols(exp_lib)


def test_spread_pipeline_rejects_depth_one():
    from e2sar_amd.dist import SpreadPipeline
    with pytest.raises(ValueError, match="depth >= 2"):
        SpreadPipeline(None, None, 1472, 16, 2, 0, depth=1)


def test_host_geometry_matches_oracle():
    from e2sar_amd import _capi
    L = _capi.lib()
    assert L.e2sar_hip_abi_version() == 1
    for v6 in (0, 1):
        assert L.e2sar_hip_total_hdr_len(v6) == O.lib().e2o_total_hdr_len(v6)
    for mtu in (65, 80, 104, 1499, 1500, 9000):
        mp = L.e2sar_hip_max_pld_len(mtu, 0)
        assert mp == O.max_pld_len(mtu)
        for b in (0, 1, mp - 1, mp, mp + 1, 1 << 20):
            assert L.e2sar_hip_num_packets(b, mp) == O.num_packets(b, mp)
    assert L.e2sar_hip_packet_stride(1436) == 1472
    assert L.e2sar_hip_packet_stride(8936) == 8976
    assert L.e2sar_hip_max_pld_len(64, 0) == 0


def test_seg_plan_host_logic():
    import ctypes as C
    from e2sar_amd import _capi
    L = _capi.lib()
    arr = (_capi.SegEvent * 4)()
    for k, b in enumerate([0, 1436, 1437, 1 << 20]):
        arr[k].bytes = b
    tot, mx = C.c_uint32(), C.c_uint32()
    assert L.e2sar_hip_seg_plan(arr, 4, 1436, C.byref(tot), C.byref(mx)) == 0
    assert [arr[k].pktBase for k in range(4)] == [0, 0, 1, 3]
    assert tot.value == 3 + 731 and mx.value == 731
    # maxPldLen 0 is a ParameterError with a message, not a crash
    assert L.e2sar_hip_seg_plan(arr, 4, 0, C.byref(tot), C.byref(mx)) == _capi.ERR_PARAMETER
    assert b"MTU" in L.e2sar_hip_last_error()


def test_no_oracle_in_product():
    # the product library must not link or embed the oracle
    from e2sar_amd import _capi
    out = subprocess.run(["nm", "-D", _capi.LIB_PATH], capture_output=True, text=True).stdout
    assert "e2o_" not in out
    for root, _, files in os.walk(os.path.join(ROOT, "e2sar_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h")):
                txt = open(os.path.join(root, f)).read()
                assert "oracle" not in txt.replace("no CPU fallback", ""), f
