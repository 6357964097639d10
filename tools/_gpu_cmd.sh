set -e
O=gpurun_out/tbl; mkdir -p $O
for r in 1 2; do for f in 2 4 8 16; do timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 20 --table-factor $f > $O/f${f}_$r.json; python -c "import json;d=json.load(open('$O/f${f}_$r.json'));print('$r factor $f',d['value'],d['roofline']['avg_launch_ms'])"; done; done
for f in 2 8; do timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 20 --table-factor $f --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 32 > $O/c3f${f}.json; python -c "import json;d=json.load(open('$O/c3f${f}.json'));print('cfg3 factor $f',d['value'],d['roofline']['avg_launch_ms'])"; done
