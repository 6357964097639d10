#!/usr/bin/env python3
"""Copy the judged summaries of a GPU evidence pass (tools/profile_round4.sh, c3_bimodal.sh,
the default bench line) from gpurun_out/ into profiles/round4/TAG/, and point the committed
PMC summaries bench.py reads (profiles/pmc_*.json) at them.
Usage: tools/collect_round4.py SRC_DIR TAG [ROUND]   (SRC_DIR e.g. gpurun_out/r4_gpu3; ROUND
default round4: the summaries go to profiles/ROUND/TAG/)"""
import csv
import json
import os
import shutil
import statistics as st
import sys

src, tag = sys.argv[1], sys.argv[2]
rnd = sys.argv[3] if len(sys.argv) > 3 else "round4"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles", rnd, tag)
os.makedirs(dst, exist_ok=True)
for f in ("bench_default.json", "bench_n2_gloo.json"):
    if os.path.exists(os.path.join(src, f)):
        shutil.copy(os.path.join(src, f), os.path.join(dst, f))
prof = os.path.join(src, "prof")
for w in sorted(os.listdir(prof)) if os.path.isdir(prof) else []:
    p = os.path.join(prof, w)
    if not os.path.isdir(p):
        continue
    o = os.path.join(dst, w)
    os.makedirs(o, exist_ok=True)
    for a, b in (("stats/run_kernel_stats.csv", "kernel_stats.csv"), ("pmc_summary.json", "pmc_summary.json"),
                 ("bench_profiled.json", "bench_profiled.json")):
        if os.path.exists(os.path.join(p, a)):
            shutil.copy(os.path.join(p, a), os.path.join(o, b))
    pmc = os.path.join(o, "pmc_summary.json")
    if os.path.exists(pmc):
        d = json.load(open(pmc))
        d["file"] = os.path.relpath(pmc, root)
        json.dump(d, open(pmc, "w"), indent=1)
        name = {"headline": "pmc_latest.json", "mtu9000": "pmc_mtu9000.json", "config3": "pmc_config3.json",
                "cold": "pmc_cold.json"}.get(w)
        if name:
            json.dump(d, open(os.path.join(root, "profiles", name), "w"), indent=1)
c3 = os.path.join(src, "c3")
if os.path.isdir(c3):
    out = {"what": "config 3 (280 x 8 MiB @ MTU 9000, 70 events per launch) in N separate bench processes on one "
                   "box, each under rocprofv3 --kernel-trace: per-launch durations (us)", "processes": []}
    i = 1
    while os.path.exists(os.path.join(c3, f"p{i}.json")):
        d = json.loads(open(os.path.join(c3, f"p{i}.json")).read().strip().splitlines()[-1])
        rows = list(csv.DictReader(open(os.path.join(c3, f"p{i}", "run_kernel_trace.csv"))))
        per = {}
        for r in rows:
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("e2sar_amd::", "")
            if k.startswith(("reas_", "seg_")):
                per.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        out["processes"].append({"value": d["value"], "kernels": {
            k: {"n": len(v), "median": round(st.median(v), 2), "min": round(min(v), 2), "max": round(max(v), 2)}
            for k, v in per.items()}})
        i += 1
    json.dump(out, open(os.path.join(dst, "config3_processes.json"), "w"), indent=1)
    if os.path.exists(os.path.join(c3, "smi.log")):
        shutil.copy(os.path.join(c3, "smi.log"), os.path.join(dst, "config3_smi.log"))
print(dst)
