set -e
E2SAR_HIP_LIB=$GRAFT_REPO_ROOT/build/variants/lib_zc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/zc_pytest.log 2>&1 || { tail -30 gpurun_out/zc_pytest.log; exit 1; }
tail -1 gpurun_out/zc_pytest.log
for r in 1 2 3; do bash tools/ab_variants.sh ab_zc_$r "--steps 20" base zc; bash tools/ab_variants.sh ab_zc9_$r "--steps 20 --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 32" base zc; done
for r in 1 2 3; do for v in base zc; do python -c "import json;d=json.load(open('gpurun_out/ab_zc_$r/$v.json'));e=json.load(open('gpurun_out/ab_zc9_$r/$v.json'));print('$r $v',d['value'],d['roofline']['avg_launch_ms']['reas_kernel'],'| 8M',e['value'],e['roofline']['avg_launch_ms']['reas_kernel'])"; done; done
