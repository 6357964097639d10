set -e
O=gpurun_out/cfg4; mkdir -p $O
run() { n=$1; shift; timeout -k 10 200 python bench.py --cpu-seconds 0 "$@" > $O/$n.json; python -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['config']['verified_roundtrip'],d['roofline']['avg_launch_ms'])"; }
run mtu1500_1m_lbv3 --lb-version 3
run mtu9000_1m --mtu 9000
run mtu9000_8m_b32 --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 32
run mtu9000_8m_b24 --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 24
run mtu1500_1m_spread_landing --landing spread
run mtu1500_1m_perf_payload --payload perf
