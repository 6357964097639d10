"""bench.py's CPU-side pieces on the CPU: argument defaults (the driver's contract) and the
cpu_baseline leg (the oracle on host threads, a tiny budget here)."""
import argparse
import os
import sys

import bench

ROOT = bench.ROOT


def test_defaults_are_the_headline_workload(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.gpus, a.mtu, a.event_bytes, a.events, a.batch_events, a.lb_version) == (1, 1500, 1 << 20, 1024, 205, 2)
    assert a.reas == "fused" and a.landing == "own" and a.payload == "random" and not a.eager


def test_cpu_baseline_reports_the_contract_fields(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    args = argparse.Namespace(event_bytes=65536, mtu=1500, lb_version=2)
    r = bench.cpu_baseline(args, 0.2)
    assert r["unit"] == "GiB/s" and r["kind"] == "port" and r["value"] > 0
    assert 1 <= r["cores"] <= 2 and r["single_core"]["cores"] == 1 and r["single_core"]["value"] > 0
    assert "MTU 1500" in r["sample"]
    a = r["all_cores"]
    assert a["cores"] == bench.host_cpu_info()["allowed"] and a["value"] > 0


def test_gpus_n_starts_one_rank_per_gpu(monkeypatch):
    # `python bench.py --gpus 2` with no launcher: bench starts torch.distributed.run with
    # 2 ranks as a child process and exits with its status (nothing touches the GPU first)
    calls = []
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "4"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd, env=None: calls.append((cmd, env)) or 7)
    try:
        bench.main()
    except SystemExit as e:
        assert e.code == 7
    else:
        raise AssertionError("bench.main() did not exit with the launcher's status")
    (cmd, env), = calls
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == [bench.os.path.abspath(bench.__file__), "--gpus", "2", "--steps", "4"][-4:]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_graph_steps_divides_the_timed_steps():
    # the whole timed region in one graph up to 64 steps, else the largest divisor <= 64
    for steps, g in ((20, 20), (10, 10), (7, 7), (5, 5), (64, 64), (100, 50), (200, 50), (67, 1), (130, 26)):
        assert bench.graph_steps(bench.parse(["--steps", str(steps)])) == g
        assert steps % g == 0
    assert bench.graph_steps(bench.parse(["--steps", "6", "--graph-steps", "3"])) == 3


def test_cpu_info_fields():
    info = bench.host_cpu_info()
    assert info["nproc"] >= 1 and 1 <= info["allowed"] <= info["nproc"]


def test_config1_cpu_loopback_runs():
    # BASELINE config 1 (the oracle's SAR path over UDP loopback, one sender + one receiver
    # thread) as bench.py's cpu_baseline leg runs it: events flow and arrive intact
    import json
    import subprocess
    exe = os.path.join(ROOT, "oracle", "build", "e2o_loopback")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    out = subprocess.run([exe, "65536", "1500", "1"], capture_output=True, text=True, timeout=60, check=True)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["events"] > 0 and res["bad_events"] == 0 and res["GiBps"] > 0


def test_abandoned_sub_leg_prints_one_line_and_exits_nonzero(tmp_path):
    """A sub-leg that fails or stalls at N > 1: rank 0 prints the run's line once (the
    headline plus the sub-leg's error), even when the deadline timer's thread and the main
    thread both reach the print, and the process exits with status 3 so torchrun / CI see it."""
    import json
    import subprocess
    prog = tmp_path / "abandon.py"
    prog.write_text(
        "import sys, threading\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import bench\n"
        "line = {'metric': 'm', 'value': 1.0}\n"
        "bench._print_line(line)\n"                       # the main thread printed already
        "t = threading.Thread(target=bench._abandon_sub_leg, args=(line, 'spread', 0, 'stalled'))\n"
        "t.start(); t.join()\n")
    r = subprocess.run([sys.executable, str(prog)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3, (r.returncode, r.stderr[-500:])
    out = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(out) == 1 and json.loads(out[0]) == {"metric": "m", "value": 1.0}
    assert "sub-leg spread abandoned (stalled)" in r.stderr
    prog2 = tmp_path / "abandon2.py"
    prog2.write_text(
        f"import sys\nsys.path.insert(0, {ROOT!r})\nimport bench\n"
        "bench._abandon_sub_leg({'metric': 'm', 'value': 2.0}, 'spread', 0, 'RuntimeError: x')\n")
    r = subprocess.run([sys.executable, str(prog2)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3
    assert json.loads(r.stdout.strip()) == {"metric": "m", "value": 2.0, "spread": {"error": "RuntimeError: x"}}
