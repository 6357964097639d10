#!/bin/bash
# Run bench.py once per environment setting.  Usage: tools/ab_env.sh TAG "bench args" "NAME:VAR=V,VAR=V" ...
# (a setting with no VAR after the colon runs the default build and environment)
set -e
TAG=$1; ARGS=$2; shift 2
mkdir -p gpurun_out/$TAG
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}
  env $(echo "$vars" | tr ',' ' ') timeout -k 10 200 python bench.py --cpu-seconds 0 $ARGS > gpurun_out/$TAG/$name.json 2> gpurun_out/$TAG/$name.err
done
for spec in "$@"; do
  name=${spec%%:*}
  python - gpurun_out/$TAG/$name.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d.get("reas_cold") or {}
print(sys.argv[1].split("/")[-1], d["value"], d["roofline"]["avg_launch_ms"], c.get("value"), (c.get("roofline") or {}).get("all_launch_ms"))
PY
done
