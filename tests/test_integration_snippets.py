"""INTEGRATION.md sections 3 and 4: every C++ snippet compiles against include/e2sar_hip.h.

The snippets are what a maintainer would paste into the reference (its SendThreadState::
_send, its receive body, its pybind module); the reference's own EventQueueItem and
enqueue are replaced by two-line stand-ins declared here.
"""
import os
import re
import subprocess
import sysconfig

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRELUDE = """#include <cstddef>
#include <cstdint>
#include <sys/types.h>
struct EventQueueItem { u_int8_t *event = nullptr; size_t bytes = 0; uint64_t eventNum = 0; uint16_t dataId = 0; };
void enqueue(EventQueueItem *item);
"""


def _snippets(section="## 3.", end="## 4."):
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        text = f.read()
    sec = text[text.index(section):(text.index(end) if end else len(text))]
    return re.findall(r"```cpp\n(.*?)```", sec, re.S)


def test_integration_has_the_three_seams():
    snips = _snippets()
    assert len(snips) == 3
    assert "e2sar_hip_seg_plan(&ev, 1, maxPldLen, &n, &maxPk)" in snips[0]


ALL = _snippets() + _snippets("## 4.", None)


@pytest.mark.parametrize("k", range(len(ALL)))
def test_integration_snippet_compiles(tmp_path, k):
    code = ALL[k]
    src = tmp_path / f"snippet{k}.cpp"
    src.write_text(PRELUDE + code)
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", "-Wno-unused-function",
           "-I", os.path.join(ROOT, "include"), str(src)]
    if "pybind11" in code:
        import pybind11
        cmd[1:1] = ["-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"]]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
