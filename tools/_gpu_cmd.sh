set -e
O=gpurun_out/bsweep; mkdir -p $O
for r in 1 2; do for b in 180 192 205 216 228; do timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 20 --batch-events $b > $O/b${b}_$r.json; python -c "import json;d=json.load(open('$O/b${b}_$r.json'));print('$r b$b',d['value'],d['roofline']['avg_launch_ms'])"; done; done
