set -e
O=gpurun_out/r3s3_range; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in base norange base; do
  if [ $v = base ]; then L=$GRAFT_REPO_ROOT/e2sar_amd/lib/libe2sar_hip.so; else L=$GRAFT_REPO_ROOT/build/variants/lib_$v.so; fi
  E2SAR_HIP_LIB=$L timeout -k 10 120 python tools/place_probe.py --trials 3 --offsets-mib 0 --shifts-mib 0 --split >> $O/probe_$v.jsonl 2> $O/probe_$v.err || { tail -20 $O/probe_$v.err; exit 1; }
  echo $v; tail -1 $O/probe_$v.jsonl
done
tools/ab_variants.sh r3s3_range_b "--subs config3" base norange
for f in gpurun_out/r3s3_range_b/*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; c=d['reas_cold']; c3=d['config3']
print('$f', d['value'], r['avg_launch_ms'], 'cold', c['value'], c['roofline']['all_launch_ms'], 'c3', c3['value'], c3['roofline']['avg_launch_ms'])"; done
