#!/bin/bash
# fused reassembly: 640 threads, and rounds 0+1 in flight during classification (EARLY), vs
# the 768/512 default; two-lane pipelines on the new kernel (repository root)
set -o pipefail
O=gpurun_out/r4_gpu17
mkdir -p $O
one() {  # name lib "args" rep
  local L=$(pwd)/e2sar_amd/lib/libe2sar_hip.so
  [ "$2" != base ] && L=$(pwd)/build/variants/lib_$2.so
  E2SAR_HIP_LIB=$L timeout -k 10 200 python bench.py --cpu-seconds 0 --cold-steps 0 --subs none $3 > $O/$1_$4.json 2> $O/$1_$4.err || { echo "$1 failed"; tail -5 $O/$1_$4.err; exit 1; }
  python3 - $O/$1_$4.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1].split("/")[-1], d["value"], r["avg_launch_ms"], r["frac"], flush=True)
PY
}
for rep in 1 2 3; do
  one h_base base "" $rep || exit 1
  one h_t640 t640 "" $rep || exit 1
  one h_t640e t640e "" $rep || exit 1
  one h_lanes2 base "--lanes 2 --batch-events 103" $rep || exit 1
  one m_base base "--mtu 9000" $rep || exit 1
  one m_t512e t512e "--mtu 9000" $rep || exit 1
  one m_t640 t640 "--mtu 9000" $rep || exit 1
done
