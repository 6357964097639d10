set -e
E2SAR_HIP_LIB=$GRAFT_REPO_ROOT/build/variants/lib_cf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cf_pytest.log 2>&1 || { tail -30 gpurun_out/cf_pytest.log; exit 1; }
tail -1 gpurun_out/cf_pytest.log
for r in 1 2 3; do bash tools/ab_variants.sh ab_cf_$r "--steps 20" base cf cf0 cf12; done
for r in 1 2 3; do for v in base cf cf0 cf12; do python -c "import json;d=json.load(open('gpurun_out/ab_cf_$r/$v.json'));print('$r $v',d['value'],d['roofline']['avg_launch_ms']['reas_kernel'])"; done; done
for v in trace trace_cf; do E2SAR_HIP_LIB=$GRAFT_REPO_ROOT/build/variants/lib_$v.so timeout -k 10 200 python tools/trace_reas.py > gpurun_out/tr2_$v.json; python -c "
import json;d=json.load(open('gpurun_out/tr2_$v.json'))['reas'];print('$v',d['classify_q']);print(d['first_wave_detail'])"; done
