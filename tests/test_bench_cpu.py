"""bench.py's CPU-side pieces on the CPU: argument defaults (the driver's contract) and the
cpu_baseline leg (the oracle on host threads, a tiny budget here)."""
import argparse
import sys

import bench


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
