#!/bin/bash
# small-slot fused reas_kernel occupancy on the headline: 768 threads at 1 workgroup per CU
# (sm1, dynamic LDS 80000) and 512 threads at 2 per CU (t512s2) vs the default 768 at 2;
# jumbo group balance on the capped occupancy (jb)
set -o pipefail
O=gpurun_out/r4_gpu33
mkdir -p $O
tools/ab_libs.sh r4_gpu33/h 3 "" base sm1 t512s2 > $O/h.log 2>&1 || { echo "h failed"; cat $O/h.log; exit 1; }
cat $O/h.log
# jumbo launch balanced on its capped occupancy (jb) vs on the uncapped one (default), MTU 9000
tools/ab_libs.sh r4_gpu33/m 2 "--mtu 9000" base jb > $O/m.log 2>&1 || { echo "m failed"; cat $O/m.log; exit 1; }
cat $O/m.log
