#!/bin/bash
# CPU baseline (oracle on host threads) at 4 / 16 / 64 events of 1 MiB per thread: shows the
# 1-thread rate running from L3 and the multi-thread rate from DRAM.
mkdir -p gpurun_out/r2i
for ev in 4 16 64; do
  E2SAR_CPU_EVENTS=$ev timeout -k 10 120 python -c "
import argparse, json, os, sys
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import bench
a = argparse.Namespace(event_bytes=1 << 20, mtu=1500, lb_version=2)
r = bench.cpu_baseline(a, 5.0)
print(json.dumps({'events_per_thread': $ev, 'T': r['cores'], 'multi': r['value'], 'single': r['single_core']['value'], 'host': r['host']}))
" >> gpurun_out/r2i/cpu_events.jsonl
done
