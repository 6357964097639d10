#!/bin/bash
# Same-box A/B of the round-2 head (8a910a1, built under build/ab_r2 by
#   mkdir -p build/ab_r2 && git archive 8a910a1 | tar -x -C build/ab_r2 && make -C build/ab_r2 all)
# against this tree: headline only (no sub-legs, no cold leg, no CPU baseline), alternating.
# Usage: tools/ab_round2_head.sh TAG [REPS]
set -e
TAG=$1; REPS=${2:-3}
O=gpurun_out/$TAG
mkdir -p $O
HERE=$(pwd)
for i in $(seq 1 $REPS); do
  (cd build/ab_r2 && timeout -k 10 200 python bench.py --cpu-seconds 0 --cold-steps 0 --quiet) \
      > $O/r2_$i.json 2> $O/r2_$i.err || { tail -20 $O/r2_$i.err; exit 1; }
  timeout -k 10 200 python bench.py --cpu-seconds 0 --cold-steps 0 --subs "" --quiet \
      > $O/head_$i.json 2> $O/head_$i.err || { tail -20 $O/head_$i.err; exit 1; }
  python - $O/r2_$i.json $O/head_$i.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("roofline") or {}
    print(f.split("/")[-1], d["value"], r.get("kernel"), r.get("avg_launch_ms"), r.get("frac"))
PY
done
