#!/bin/bash
# fused kernel held to 64 VGPRs (8 waves per SIMD; 32 B/lane of spills): 1024 threads (two
# workgroups of 16 waves per CU) and 512 threads (four of 8) vs the 768/512 default (repository root)
set -o pipefail
O=gpurun_out/r4_gpu25
mkdir -p $O
tools/ab_libs.sh r4_gpu25/h 3 "" base t1024w8 t512w8 > $O/h.log 2>&1 || { echo "h failed"; cat $O/h.log; exit 1; }
cat $O/h.log
tools/ab_libs.sh r4_gpu25/m 2 "--mtu 9000" base t1024w8 t512w8 > $O/m.log 2>&1 || { echo "m failed"; cat $O/m.log; exit 1; }
cat $O/m.log
