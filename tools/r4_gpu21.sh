#!/bin/bash
# pipelined scatter+classify (cold leg): classify waves at priority 3, at 75 % (cp3), at the
# front (cp3a0) and half way (cp3a50) of the grid, vs the default (repository root)
set -o pipefail
O=gpurun_out/r4_gpu21
mkdir -p $O
run() {  # tag "args" libs...
  local t=$1 a=$2; shift 2
  tools/ab_libs.sh r4_gpu21/$t 2 "$a" "$@" > $O/$t.log 2>&1 || { echo "$t failed"; cat $O/$t.log; exit 1; }
  echo "== $t ($a)"
  for f in $O/$t/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d.get('reas_cold')
print('  cold', '$f'.split('/')[-1], c['value'], c['roofline']['avg_launch_ms'], c['roofline']['frac']) if c else None"; done
}
run cold1500 "--cold-steps 10" base cp3 cp3a0 cp3a50
run cold9000 "--mtu 9000 --cold-steps 10" base cp3 cp3a0
tools/ab_libs.sh r4_gpu21/c3 2 "--mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70" base fusedbig > $O/c3.log 2>&1 || { echo "c3 failed"; cat $O/c3.log; exit 1; }
echo "== c3 (fused 512-thread kernel on config 3's 590 MB batches)"; cat $O/c3.log
