#!/usr/bin/env python3
"""Print the key numbers of bench.py JSON lines: tools/summ.py FILE..."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    r = d["roofline"]
    print(f"{f}: value {d['value']} ms/step {d['ms_per_step']} dom {r['kernel']} frac {r['frac']} "
          f"launch_ms {r['avg_launch_ms']} copy {r.get('copy_GBps')}")
    for k in ("mtu9000", "config3", "reas_cold"):
        v = d.get(k)
        if v:
            rr = v.get("roofline") or {}
            print(f"   {k}: {v.get('value')} verified {v.get('verified')} {rr.get('kernel')} frac {rr.get('frac')} "
                  f"{rr.get('avg_launch_ms') or rr.get('all_launch_ms')}")
    if d.get("spread"):
        print("   spread", d["spread"].get("foreign_sent_per_step"), d["spread"].get("received_per_step"))
    if d.get("cpu_baseline"):
        print("   cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
