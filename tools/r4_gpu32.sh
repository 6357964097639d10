#!/bin/bash
# reas_kernel occupancy caps by dynamic LDS: small-slot launch at 2 workgroups per CU (sm2)
# on the headline; jumbo launch at 2 (j2) and 3 (j3) per CU at MTU 9000 (repository root)
set -o pipefail
O=gpurun_out/r4_gpu32
mkdir -p $O
tools/ab_libs.sh r4_gpu32/h 3 "" base sm2 > $O/h.log 2>&1 || { echo "h failed"; cat $O/h.log; exit 1; }
cat $O/h.log
tools/ab_libs.sh r4_gpu32/m 2 "--mtu 9000" base j2 j3 > $O/m.log 2>&1 || { echo "m failed"; cat $O/m.log; exit 1; }
cat $O/m.log
