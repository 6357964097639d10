#!/bin/bash
# scatter geometry A/B on config 3 and the cold leg (inside build/snap)
set -o pipefail
O=gpurun_out/r4_gpu7
mkdir -p $O
ROOTDIR=$(cd ../.. && pwd)
ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu7/c3 2 "--mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70" base su3 su5 su6 > $O/c3.log 2>&1 || { echo "c3 failed"; cat $O/c3.log; exit 1; }
cat $O/c3.log
ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu7/cold 2 "--cold-steps 10" base su3 sg11 > $O/cold.log 2>&1 || { echo "cold failed"; cat $O/cold.log; exit 1; }
cat $O/cold.log
for f in $O/cold/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['reas_cold']; print('$f'.split('/')[-1], c['value'], c['roofline']['avg_launch_ms'], c['roofline']['frac'])"; done
