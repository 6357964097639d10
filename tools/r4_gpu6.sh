#!/bin/bash
# lookup-first A/B + trace + GPU suite (inside build/snap)
set -o pipefail
O=gpurun_out/r4_gpu6
mkdir -p $O
ROOTDIR=$(cd ../.. && pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 || { echo "parity failed"; tail -30 $O/pytest_parity.log; exit 1; }
tail -2 $O/pytest_parity.log
ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu6/lf 3 "" base lf0 rf > $O/lf.log 2>&1 || { echo "lf failed"; cat $O/lf.log; exit 1; }
cat $O/lf.log
E2SAR_HIP_LIB=$ROOTDIR/build/variants/lib_trace.so timeout -k 10 120 python tools/trace_reas.py > $O/trace.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
E2SAR_RANDOM_SEEDS=60 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k random -x -q --timeout 300 --timeout-method thread > $O/pytest_random60.log 2>&1; echo "random rc=$?"; tail -2 $O/pytest_random60.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -3 $O/pytest.log
