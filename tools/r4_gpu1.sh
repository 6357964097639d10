#!/bin/bash
# Round 4, first GPU pass (run inside build/snap via tools/gpu_snap_run.sh):
# same-box A/B of round 2 vs this tree, the GPU suite, the A/B-only forms against their
# variant library, and the two-rank spread rehearsal (gloo, both ranks on GPU 0).
set -o pipefail
O=gpurun_out/r4_gpu1
mkdir -p $O
timeout -k 10 120 ../../build/ubench_rounds 210 15 > $O/ubench_rounds.json 2> $O/ubench_rounds.err || { echo "ubench failed"; cat $O/ubench_rounds.err; exit 1; }
cat $O/ubench_rounds.json
ROOTDIR=$(cd ../.. && pwd) tools/ab_libs.sh r4_gpu1/all 2 "" base all5 all3 all4 > $O/all.log 2>&1 || { echo "all failed"; tail -20 $O/all.log; exit 1; }
cat $O/all.log
tools/ab_round2_head.sh r4_gpu1/ab 3 > $O/ab.log 2>&1 || { echo "ab failed"; tail -20 $O/ab.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
E2SAR_HIP_LIB=build/variants/lib_experimental.so timeout -k 10 300 python -u -m pytest tests/test_gpu_chained.py tests/test_gpu_xcd_groups.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exp.log 2>&1 || { echo "exp failed"; tail -30 $O/pytest_exp.log; exit 1; }
E2SAR_BENCH_BACKEND=gloo E2SAR_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --cpu-seconds 0 --cold-steps 0 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { echo "n2 failed"; tail -30 $O/bench_n2_gloo.err; exit 1; }
echo done
