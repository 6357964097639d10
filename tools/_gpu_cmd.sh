set -e
tools/ab_variants.sh r3s3_sc "--subs config3" base su8 su8g3 su5g2 g2
cp gpurun_out/r3s3_sc/base.json gpurun_out/r3s3_sc/base1.json
tools/ab_variants.sh r3s3_sc "--subs config3" base
for f in gpurun_out/r3s3_sc/*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; c=d['reas_cold']; c3=d['config3']
print('$f', d['value'], r['avg_launch_ms'], 'cold', c['value'], c['roofline']['all_launch_ms'], 'c3', c3['value'], c3['roofline']['avg_launch_ms'])"; done
