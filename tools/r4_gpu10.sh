#!/bin/bash
# staged scatter stores as the default: GPU suite, then A/B against never staging (inside build/snap)
set -o pipefail
O=gpurun_out/r4_gpu10
mkdir -p $O
ROOTDIR=$(cd ../.. && pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu10/c3 2 "--mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70" base nostage > $O/c3.log 2>&1 || { echo "c3 failed"; cat $O/c3.log; exit 1; }
cat $O/c3.log
