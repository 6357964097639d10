#!/bin/bash
# reas_kernel occupancy caps by dynamic LDS, tree default = jumbo launch at 2 per CU:
# small-slot launch at 2 per CU (sm2) on the headline; jumbo uncapped (j0) and at 3 per CU
# (j3) at MTU 9000; then GPU suite, smoke and default bench line (repository root)
set -o pipefail
O=gpurun_out/r4_gpu32
mkdir -p $O
tools/ab_libs.sh r4_gpu32/m 2 "--mtu 9000" base j0 j3 > $O/m.log 2>&1 || { echo "m failed"; cat $O/m.log; exit 1; }
cat $O/m.log
tools/ab_libs.sh r4_gpu32/h 2 "" base sm2 > $O/h.log 2>&1 || { echo "h failed"; cat $O/h.log; exit 1; }
cat $O/h.log
E2SAR_RANDOM_SEEDS=40 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
tail -c 300 $O/bench_default.json; echo
