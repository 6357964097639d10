#!/bin/bash
# wave-0-late A/B (inside build/snap) + GPU suite on the new default
set -o pipefail
O=gpurun_out/r4_gpu5
mkdir -p $O
ROOTDIR=$(cd ../.. && pwd)
ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu5/w0 3 "" base w0early > $O/w0.log 2>&1 || { echo "w0 failed"; tail $O/w0.log; exit 1; }
cat $O/w0.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -3 $O/pytest.log
