set -e
for r in 1 2; do bash tools/ab_variants.sh ab_u_$r "--steps 20" base u3 u5 u6; done
for r in 1 2; do for v in base u3 u5 u6; do python -c "import json;d=json.load(open('gpurun_out/ab_u_$r/$v.json'));print('$r $v',d['value'],d['roofline']['avg_launch_ms'])"; done; done
