#!/bin/bash
# Interleaved A/B of library builds on one box: bench.py (headline only) once per name per
# repetition; "base" = the tree's own library, NAME = $ROOTDIR/build/variants/lib_NAME.so.
# Usage: ROOTDIR=... tools/ab_libs.sh TAG REPS "bench args" name...
TAG=$1; REPS=$2; ARGS=$3; shift 3
ROOTDIR=${ROOTDIR:-$(pwd)}
O=gpurun_out/$TAG
mkdir -p $O
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    if [ "$v" = base ]; then L=$(pwd)/e2sar_amd/lib/libe2sar_hip.so; else L=$ROOTDIR/build/variants/lib_$v.so; fi
    E2SAR_HIP_LIB=$L timeout -k 10 200 python bench.py --cpu-seconds 0 --cold-steps 0 --subs none $ARGS > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { echo "$v failed"; tail -5 $O/${v}_$rep.err; exit 1; }
    python3 - $O/${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
line = [sys.argv[1].split("/")[-1], d["value"], r["avg_launch_ms"], r["frac"]]
c = d.get("reas_cold")
if c:
    line += ["cold", c.get("value"), c.get("roofline", {}).get("avg_launch_ms"), c.get("roofline", {}).get("frac")]
print(*line)
PY
  done
done
