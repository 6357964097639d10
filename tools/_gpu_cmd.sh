set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_v2.log 2>&1 || { tail -30 gpurun_out/pytest_v2.log; exit 1; }
tail -1 gpurun_out/pytest_v2.log
O=gpurun_out/r3s3_v2; mkdir -p $O
for v in base v1 base v1; do
  if [ $v = base ]; then L=$R/e2sar_amd/lib/libe2sar_hip.so; else L=$R/build/variants/lib_$v.so; fi
  E2SAR_HIP_LIB=$L timeout -k 10 120 python tools/place_probe.py --trials 3 --offsets-mib 0 --shifts-mib 0 --split >> $O/probe_$v.jsonl 2> $O/probe_$v.err || { tail -20 $O/probe_$v.err; exit 1; }
  echo $v; tail -1 $O/probe_$v.jsonl | cut -c 100-400
done
tools/ab_variants.sh r3s3_v2b "--subs none" base v1
cp gpurun_out/r3s3_v2b/base.json gpurun_out/r3s3_v2b/base1.json; cp gpurun_out/r3s3_v2b/v1.json gpurun_out/r3s3_v2b/v11.json
tools/ab_variants.sh r3s3_v2b "--subs none" base v1
for f in gpurun_out/r3s3_v2b/*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['reas_cold']; print('$f', d['value'], 'cold', c['value'], c['roofline']['frac'], c['roofline']['all_launch_ms'])"; done
