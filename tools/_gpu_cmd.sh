set -e
for r in 1 2 3; do bash tools/ab_variants.sh ab_sa_$r "--steps 20 --no-verify" base slotarena; done
for r in 1 2 3; do for v in base slotarena; do python -c "import json;d=json.load(open('gpurun_out/ab_sa_$r/$v.json'));print('$r $v',d['value'],d['roofline']['avg_launch_ms']['reas_kernel'])"; done; done
for v in trace trace_slotarena; do E2SAR_HIP_LIB=$GRAFT_REPO_ROOT/build/variants/lib_$v.so timeout -k 10 200 python tools/trace_reas.py > gpurun_out/tr_$v.json; python -c "
import json;d=json.load(open('gpurun_out/tr_$v.json'))['reas'];print('$v',d['classify_q']);print(d['first_wave_detail'])"; done
