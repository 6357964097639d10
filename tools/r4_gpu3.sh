#!/bin/bash
# Round 4, evidence pass (inside build/snap): the driver's default bench line, isolated
# per-workload rocprof + PMC profiles, config 3's two speeds with clocks/power sampled.
set -o pipefail
O=gpurun_out/r4_gpu3
mkdir -p $O
ROOTDIR=$(cd ../.. && pwd)
ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu3/early2 2 "" base early2 > $O/early2.log 2>&1 || { echo "early2 failed"; tail $O/early2.log; exit 1; }
cat $O/early2.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
tools/profile_round4.sh $O/prof headline cold mtu9000 config3 || { echo "profile failed"; tail $O/prof/progress.log; exit 1; }
tools/c3_bimodal.sh $O/c3 5 > $O/c3.log 2>&1 || { echo "c3 failed"; tail $O/c3.log; exit 1; }
echo done
