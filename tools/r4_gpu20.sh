#!/bin/bash
# fused kernel: classifier wave priority (s_setprio 1 / 3 during classification) (repository root)
set -o pipefail
O=gpurun_out/r4_gpu20
mkdir -p $O
tools/ab_libs.sh r4_gpu20/h 3 "" base prio1 prio3 > $O/h.log 2>&1 || { echo "h failed"; cat $O/h.log; exit 1; }
cat $O/h.log
tools/ab_libs.sh r4_gpu20/m 2 "--mtu 9000" base prio3 > $O/m.log 2>&1 || { echo "m failed"; cat $O/m.log; exit 1; }
cat $O/m.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k group_sizes -x -q --timeout 120 --timeout-method thread > $O/pytest_groups.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_groups.log; exit 1; }
tail -2 $O/pytest_groups.log
