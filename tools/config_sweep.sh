#!/bin/bash
# Bench lines for BASELINE's configurations with the current code (one MI355X).
# Usage: tools/config_sweep.sh TAG
set -e
O=gpurun_out/$1; mkdir -p $O
B="timeout -k 10 240 python bench.py --cpu-seconds 0"
$B --mtu 9000 --cold-steps 0 > $O/b_1m_mtu9000.json 2> $O/b.err
$B --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70 --cold-steps 0 > $O/c_8m_mtu9000_70ev.json 2> $O/c.err
$B --mtu 9000 --event-bytes 8388608 --events 256 --batch-events 32 --cold-steps 0 > $O/c_8m_mtu9000_32ev.json 2> $O/c32.err
$B --lb-version 3 --cold-steps 0 > $O/a_lbv3.json 2> $O/v3.err
$B --landing spread --cold-steps 0 > $O/a_spread_n1.json 2> $O/spread.err
E2SAR_BENCH_BACKEND=gloo E2SAR_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --cpu-seconds 0 --cold-steps 0 > $O/a_n2_gloo_share.json 2> $O/n2.err
timeout -k 10 300 python tools/bench_hostpath.py --batch-events 64 > $O/hostpath64.json 2> $O/host.err
