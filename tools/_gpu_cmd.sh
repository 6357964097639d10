set -e
for r in 1 2; do bash tools/ab_variants.sh ab_sl_$r "--steps 20" base sl4 sl16 sl60; bash tools/ab_variants.sh ab_sl9_$r "--steps 20 --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 32" base sl4 sl16 sl60; done
for r in 1 2; do for v in base sl4 sl16 sl60; do python -c "import json;d=json.load(open('gpurun_out/ab_sl_$r/$v.json'));e=json.load(open('gpurun_out/ab_sl9_$r/$v.json'));print('$r $v',d['value'],d['roofline']['avg_launch_ms']['reas_kernel'],'| 8M',e['value'],e['roofline']['avg_launch_ms']['reas_kernel'])"; done; done
