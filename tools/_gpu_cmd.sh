set -e
O=gpurun_out/cosched; mkdir -p $O
run() { n=$1; shift; timeout -k 10 200 python bench.py --cpu-seconds 0 "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }; python -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['config']['verified_roundtrip'],d['roofline']['avg_launch_ms'])"; }
run base
run co205 --reas cosched
run co128 --reas cosched --batch-events 128
run co103 --reas cosched --batch-events 103
run co64 --reas cosched --batch-events 64
run co160 --reas cosched --batch-events 160
