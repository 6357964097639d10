#!/bin/bash
# probe: what the arena's returning atomic costs the fused kernel at 1 MiB (noar = offsets
# from the event number, a probe build, not an allocator) (repository root)
set -o pipefail
O=gpurun_out/r4_gpu19
mkdir -p $O
tools/ab_libs.sh r4_gpu19/h 3 "" base noar > $O/h.log 2>&1 || { echo "h failed"; cat $O/h.log; exit 1; }
cat $O/h.log
tools/ab_libs.sh r4_gpu19/m 2 "--mtu 9000" base noar > $O/m.log 2>&1 || { echo "m failed"; cat $O/m.log; exit 1; }
cat $O/m.log
