#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into per-launch HBM traffic for the SAR kernels.

Usage: tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json [--workload STR]

Each directory holds one `rocprofv3 --pmc <COUNTER> --kernel-trace --output-format csv`
pass (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).  Corrections follow
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads exactly half of a
wide coalesced 16-B/lane stream on gfx950, so it is doubled; WRITE_SIZE (KiB) is exact
for 16-B/lane stores.  Output: bytes per launch per kernel.
"""
import csv
import json
import sys
from collections import defaultdict


def load(d, counter):
    vals = defaultdict(list)
    with open(f"{d}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            if "e2sar_amd::" not in name:
                continue
            short = name.split("(")[0].replace("void ", "").replace("e2sar_amd::", "")
            vals[short].append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main():
    fd, wd, out = sys.argv[1:4]
    workload = None
    if "--workload" in sys.argv:
        # e.g. mtu=1500,event_bytes=1048576,batch_events=128,lb_version=2
        kv = sys.argv[sys.argv.index("--workload") + 1]
        workload = {k: int(v) for k, v in (x.split("=") for x in kv.split(","))}
    fetch = load(fd, "FETCH_SIZE")
    write = load(wd, "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, --kernel-trace",
           "correction": "FETCH_SIZE x2 (gfx950 half-count on 16-B/lane streams), WRITE_SIZE x1, KiB -> bytes",
           "workload": workload, "file": out, "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2.0 * sum(f) / len(f) if f else None
        wb = sum(w) / len(w) if w else None
        res["kernels"][k] = {"launches_fetch_pass": len(f), "launches_write_pass": len(w),
                             "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                             "hbm_bytes_per_launch": (fb or 0) + (wb or 0)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
