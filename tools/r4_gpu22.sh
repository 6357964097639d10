#!/bin/bash
# event-size sweep (five whole batches per step, ~221 MB of slots per batch) on the
# 768/512-thread fused kernel vs 256 threads, plus LB v3, spread landing at N = 1 and the
# host path on the final code (repository root)
set -o pipefail
O=gpurun_out/r4_gpu22
mkdir -p $O
one() {  # name lib "args"
  local L=$(pwd)/e2sar_amd/lib/libe2sar_hip.so
  [ "$2" != base ] && L=$(pwd)/build/variants/lib_$2.so
  E2SAR_HIP_LIB=$L timeout -k 10 200 python bench.py --cpu-seconds 0 --cold-steps 0 --subs none $3 > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -5 $O/$1.err; exit 1; }
  python3 - $O/$1.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1].split("/")[-1], d["value"], r["avg_launch_ms"], r["frac"], flush=True)
PY
}
for mtu in 1500 9000; do
  for sz in 65536:16384:3277 262144:4096:820 4194304:260:52 8388608:130:26; do
    IFS=: read b e be <<< "$sz"
    for lib in base t256; do one s_${mtu}_${b}_$lib $lib "--mtu $mtu --event-bytes $b --events $e --batch-events $be" || exit 1; done
  done
done
one lbv3 base "--lb-version 3" || exit 1
one spread_n1 base "--landing spread" || exit 1
timeout -k 10 300 python tools/bench_hostpath.py --batch-events 64 > $O/hostpath64.json 2> $O/host.err || { echo "hostpath failed"; tail -5 $O/host.err; exit 1; }
tail -c 600 $O/hostpath64.json
