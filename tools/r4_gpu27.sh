#!/bin/bash
# occupancy cap (6 workgroups per CU) for unstaged streaming scatter launches: GPU suite, A/B
# against no cap, and a fresh cold-leg profile (repository root)
set -o pipefail
O=gpurun_out/r4_gpu27
mkdir -p $O
E2SAR_RANDOM_SEEDS=40 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
run() {  # tag reps "args" libs...
  local t=$1 r=$2 a=$3; shift 3
  tools/ab_libs.sh r4_gpu27/$t $r "$a" "$@" > $O/$t.log 2>&1 || { echo "$t failed"; cat $O/$t.log; exit 1; }
  echo "== $t ($a)"; cat $O/$t.log
  for f in $O/$t/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d.get('reas_cold')
print('  cold', '$f'.split('/')[-1], c['value'], c['roofline']['avg_launch_ms'], c['roofline']['frac']) if c else None"; done
}
run cold1500 3 "--cold-steps 10" base nocap
run cold9000 2 "--mtu 9000 --cold-steps 10" base nocap
timeout -k 10 600 tools/profile_round4.sh $O/prof cold || { echo "profile failed"; cat $O/prof/progress.log; exit 1; }
cat $O/prof/progress.log
