"""Segmenter MTU rules on the CPU (e2sarDPSegmenter.cpp:56-110, hpp:307-308).

An auto-detected interface MTU above 9000 (jumbo 9216, IPoIB 65520) must be refused like
an explicit override above 9000: the reference checks the resolved MTU.  The rules are
the façade's own functions (detail::resolve_mtu / check_mtu_limit, segmenter.cpp), called
from a small program linked against libe2sar_amd.so -- no GPU call is made.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "e2sar_amd", "lib")

PROG = r"""
#include <cstdio>
#include <string>
#include "e2sar_amd/e2sar.hpp"
namespace e2sar { namespace detail {
uint32_t resolve_mtu(uint16_t flagsMtu, uint32_t ifMtu, const std::string &iface);
void check_mtu_limit(uint32_t mtu);
} }
static const char *run(unsigned flagsMtu, unsigned ifMtu)
{
    try {
        uint32_t m = e2sar::detail::resolve_mtu((uint16_t)flagsMtu, ifMtu, "ifX");
        e2sar::detail::check_mtu_limit(m);
        static char buf[32];
        snprintf(buf, sizeof buf, "ok %u", m);
        return buf;
    } catch (const e2sar::E2SARException &e) {
        static std::string s;
        s = std::string("err ") + std::string(e);
        return s.c_str();
    }
}
int main()
{
    const unsigned cases[][2] = {{0, 1500}, {0, 9000}, {0, 9216}, {0, 65520}, {0, 0},
                                 {1500, 9216}, {9000, 9216}, {9216, 65520}, {9000, 1500}, {1500, 0}};
    for (auto &c : cases) printf("%u %u %s\n", c[0], c[1], run(c[0], c[1]));
    return 0;
}
"""


def test_resolved_mtu_above_9000_is_refused(tmp_path):
    if not os.path.exists(os.path.join(LIB, "libe2sar_amd.so")):
        pytest.skip("libe2sar_amd.so not built")
    src = tmp_path / "mtu.cpp"
    src.write_text(PROG)
    exe = tmp_path / "mtu"
    r = subprocess.run(["g++", "-std=c++17", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                        "-L", LIB, "-le2sar_amd", "-le2sar_hip", f"-Wl,-rpath,{LIB}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines()
    got = {tuple(map(int, l.split()[:2])): l.split(None, 2)[2] for l in out}
    assert got[(0, 1500)] == "ok 1500"
    assert got[(0, 9000)] == "ok 9000"
    assert got[(0, 9216)].startswith("err") and "limit 9000" in got[(0, 9216)]
    assert got[(0, 65520)].startswith("err") and "limit 9000" in got[(0, 65520)]
    assert "reported as 0" in got[(0, 0)]
    assert got[(1500, 9216)] == "ok 1500"
    assert got[(9000, 9216)] == "ok 9000"
    assert "limit 9000" in got[(9216, 65520)]
    assert "exceeds outgoing interface MTU" in got[(9000, 1500)]
    assert got[(1500, 0)] == "ok 1500"


NUMBERING = r"""
#include <atomic>
#include <cstdio>
#include "e2sar_amd/e2sar.hpp"
namespace e2sar { namespace detail {
EventNum_t take_send_number(std::atomic<EventNum_t> &userEventNum, EventNum_t eventNum, size_t depth, size_t cap,
                            bool *accepted);
} }
int main()
{
    // a send queue of capacity 3 (the facade's is 2047, e2sarDPSegmenter.hpp:101)
    std::atomic<e2sar::EventNum_t> num{0};
    size_t depth = 0;
    auto push = [&](e2sar::EventNum_t ev) {
        bool ok;
        const auto n = e2sar::detail::take_send_number(num, ev, depth, 3, &ok);
        if (ok) depth++;
        printf("%llu %d\n", (unsigned long long)n, ok ? 1 : 0);
    };
    push(0); push(0); push(0);        // 0 1 2 queued
    push(0);                          // 3 refused: the number is consumed anyway
    depth--;                          // the send thread takes one
    push(0);                          // 4 queued: 3 is a gap
    push(0);                          // 5 refused
    depth = 0;
    push(100);                        // explicit number resets the counter
    push(0);                          // 101
    return 0;
}
"""


def test_send_queue_numbering_under_a_full_queue(tmp_path):
    """addToSendQueue takes userEventNum++ before the push can fail (e2sarDPSegmenter.cpp:
    937 before 939-946), so a refused default-numbered event leaves a gap in the numbering;
    an explicit event number resets the counter first (cpp:926-927)."""
    if not os.path.exists(os.path.join(LIB, "libe2sar_amd.so")):
        pytest.skip("libe2sar_amd.so not built")
    src = tmp_path / "num.cpp"
    src.write_text(NUMBERING)
    exe = tmp_path / "num"
    r = subprocess.run(["g++", "-std=c++17", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                        "-L", LIB, "-le2sar_amd", "-le2sar_hip", f"-Wl,-rpath,{LIB}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = [tuple(map(int, l.split())) for l in
           subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines()]
    assert out == [(0, 1), (1, 1), (2, 1), (3, 0), (4, 1), (5, 0), (100, 1), (101, 1)]
