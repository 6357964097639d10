set -e
for r in 1 2; do
tools/ab_variants.sh r3s3_cls2_$r "--subs none" base cls65 cls75 cls80
done
for f in gpurun_out/r3s3_cls2_*/*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; c=d['reas_cold']
print('$f', d['value'], 'cold', c['value'], c['roofline']['frac'], c['roofline']['all_launch_ms'])"; done
