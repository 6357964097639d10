set -e
O=gpurun_out/c3g3; mkdir -p $O
for r in 1 2 3; do for g in 0 24 32 40; do
  if [ $g = 0 ]; then unset E2SAR_REAS_G; else export E2SAR_REAS_G=$g; fi
  timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 30 --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 32 > $O/g${g}_$r.json
  python -c "import json;d=json.load(open('$O/g${g}_$r.json'));print('$r G $g',d['value'],d['roofline']['avg_launch_ms'])"
done; done
