#!/bin/bash
# LDS-staged aligned scatter stores (sh3) on every scatter user (inside build/snap)
set -o pipefail
O=gpurun_out/r4_gpu9
mkdir -p $O
ROOTDIR=$(cd ../.. && pwd)
run() {  # tag "args"
  ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu9/$1 2 "$2" base sh3 > $O/$1.log 2>&1 || { echo "$1 failed"; cat $O/$1.log; exit 1; }
  cat $O/$1.log
  for f in $O/$1/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d.get('reas_cold')
print('  cold', '$f'.split('/')[-1], c['value'], c['roofline']['avg_launch_ms'], c['roofline']['frac']) if c else None"; done
}
run cold1500 "--cold-steps 10"
run cold9000 "--mtu 9000 --cold-steps 10"
run ro "--reference-order"
run split "--reas split"
