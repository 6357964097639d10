#!/bin/bash
# scatter / pipelined scatter+classify occupancy caps (dynamic LDS: p6 / p5 / p4 = at most
# 6 / 5 / 4 workgroups per CU instead of 8) on the cold legs and config 3 (repository root)
set -o pipefail
O=gpurun_out/r4_gpu26
mkdir -p $O
run() {  # tag "args" libs...
  local t=$1 a=$2; shift 2
  tools/ab_libs.sh r4_gpu26/$t 2 "$a" "$@" > $O/$t.log 2>&1 || { echo "$t failed"; cat $O/$t.log; exit 1; }
  echo "== $t ($a)"; cat $O/$t.log
  for f in $O/$t/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d.get('reas_cold')
print('  cold', '$f'.split('/')[-1], c['value'], c['roofline']['avg_launch_ms'], c['roofline']['frac']) if c else None"; done
}
run cold1500 "--cold-steps 10" base p6 p5 p4
run cold9000 "--mtu 9000 --cold-steps 10" base p6 p4
run c3 "--mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70" base p6 p4
