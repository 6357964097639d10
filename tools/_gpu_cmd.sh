set -e
E2SAR_HIP_LIB=$GRAFT_REPO_ROOT/build/variants/lib_s128.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s128_pytest.log 2>&1 || { tail -30 gpurun_out/s128_pytest.log; exit 1; }
tail -1 gpurun_out/s128_pytest.log
for r in 1 2 3; do bash tools/ab_variants.sh ab_s128_$r "--steps 20" base s128; done
for r in 1 2 3; do for v in base s128; do python -c "import json;d=json.load(open('gpurun_out/ab_s128_$r/$v.json'));print('$r $v',d['value'],d['roofline']['avg_launch_ms']['reas_kernel'])"; done; done
