"""Every gfx950 kernel compiles without scratch (private-memory) traffic or register spills.

A struct left in scratch halved seg_kernel's rate once (a reference into a by-value
struct kept the whole struct in private memory: 48 B/lane of scratch loads per round);
the compiler's resource remarks catch that on the CPU, before any GPU run.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
SOURCES = ["e2sar_amd/csrc/sar_kernels.hip"]


def _remarks(src, tmp_path):
    out = tmp_path / (os.path.basename(src) + ".o")
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only",
                        "-Iinclude", "-Ie2sar_amd/csrc", "-c", src, "-o", str(out),
                        "-Rpass-analysis=kernel-resource-usage"],
                       cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    kernels, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = kernels.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+) \[", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    return kernels


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc absent")
@pytest.mark.parametrize("src", SOURCES)
def test_no_scratch_no_spills(src, tmp_path):
    kernels = _remarks(src, tmp_path)
    assert kernels, "no kernel resource remarks parsed"
    bad = {k: v for k, v in kernels.items()
           if v.get("ScratchSize", 0) or v.get("VGPRs Spill", 0) or v.get("SGPRs Spill", 0)}
    assert not bad, f"kernels with scratch or spills: {bad}"
