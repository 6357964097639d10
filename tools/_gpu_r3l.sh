set -e
O=gpurun_out/r3l; mkdir -p $O
tools/ab_variants.sh r3l/a "--subs none --cold-steps 0" base srcal srcal_nopipe
tools/ab_variants.sh r3l/b "--subs none --cold-steps 0" base srcal srcal_nopipe
E2SAR_HIP_LIB=$GRAFT_REPO_ROOT/build/variants/lib_srcal.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_srcal.log 2>&1
