set -e
O=gpurun_out/segu; mkdir -p $O
tools/ab_variants.sh segu "--steps 20" base s2 s6 s8 base s8
for v in base s2 s6 s8; do python -c "import json;d=json.load(open('$O/$v.json'));print('$v',d['value'],d['roofline']['avg_launch_ms'])"; done
