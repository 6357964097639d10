#!/bin/bash
# staged chunk-range scatter (E2SAR_SCATTER_RANGE=2): GPU parity suite on that build, then A/B (inside build/snap)
set -o pipefail
O=gpurun_out/r4_gpu11
mkdir -p $O
ROOTDIR=$(cd ../.. && pwd)
E2SAR_HIP_LIB=$ROOTDIR/build/variants/lib_range2.so E2SAR_RANDOM_SEEDS=40 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_range2.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_range2.log; exit 1; }
tail -2 $O/pytest_range2.log
run() {  # tag "args"
  ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu11/$1 2 "$2" base range2 > $O/$1.log 2>&1 || { echo "$1 failed"; cat $O/$1.log; exit 1; }
  cat $O/$1.log
  for f in $O/$1/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d.get('reas_cold')
print('  cold', '$f'.split('/')[-1], c['value'], c['roofline']['avg_launch_ms'], c['roofline']['frac']) if c else None"; done
}
run c3 "--mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70"
run cold9000 "--mtu 9000 --cold-steps 10"
run split "--reas split"
run ro "--reference-order"
