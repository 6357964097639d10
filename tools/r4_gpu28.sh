#!/bin/bash
# seg_kernel occupancy caps by dynamic LDS (s7 / s6 / s5 = at most 7 / 6 / 5 workgroups per
# CU instead of 8), headline and MTU 9000 (repository root)
set -o pipefail
O=gpurun_out/r4_gpu28
mkdir -p $O
tools/ab_libs.sh r4_gpu28/h 3 "" base s7 s6 s5 > $O/h.log 2>&1 || { echo "h failed"; cat $O/h.log; exit 1; }
cat $O/h.log
tools/ab_libs.sh r4_gpu28/m 2 "--mtu 9000" base s6 > $O/m.log 2>&1 || { echo "m failed"; cat $O/m.log; exit 1; }
cat $O/m.log
tools/ab_libs.sh r4_gpu28/c3 2 "--mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70" base s6 > $O/c3.log 2>&1 || { echo "c3 failed"; cat $O/c3.log; exit 1; }
cat $O/c3.log
