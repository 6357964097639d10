#!/bin/bash
# Run bench.py once per argument set (no CPU baseline), each under its own time limit.
# Usage: tools/ab_args.sh TAG "name|bench args" ...   (a name may repeat: runs are numbered)
set -e
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
i=0
for spec in "$@"; do
  i=$((i + 1))
  name=${spec%%|*}; args=${spec#*|}
  [ "$args" = "$spec" ] && args=""
  timeout -k 10 200 python bench.py --cpu-seconds 0 $args > $O/${i}_$name.json 2> $O/${i}_$name.err || { tail -20 $O/${i}_$name.err; exit 1; }
  python - $O/${i}_$name.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
c = d.get("reas_cold") or {}
subs = {k: v.get("value") for k, v in d.items() if isinstance(v, dict) and "value" in v and k not in ("cpu_baseline",)}
print(sys.argv[1].split("/")[-1], d["value"], r.get("kernel"), r.get("avg_launch_ms"), r.get("frac"), subs)
PY
done
