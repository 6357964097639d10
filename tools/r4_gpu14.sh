#!/bin/bash
# fused reassembly: workgroup size x group size, interleaved on one box (repository root)
set -o pipefail
O=gpurun_out/r4_gpu14
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
for rep in 1 2; do
  one h_base base "" $rep || exit 1
  one h_t512 t512 "" $rep || exit 1
  one h_t512_g44 t512 "--reas-group 44" $rep || exit 1
  one h_t512_g33 t512 "--reas-group 33" $rep || exit 1
  one h_t512_g22 t512 "--reas-group 22" $rep || exit 1
  one h_t768 t768 "" $rep || exit 1
  one h_t768_g64 t768 "--reas-group 64" $rep || exit 1
  one h_t768_g33 t768 "--reas-group 33" $rep || exit 1
  one m_base base "--mtu 9000" $rep || exit 1
  one m_t512 t512 "--mtu 9000" $rep || exit 1
  one m_t512_g11 t512 "--mtu 9000 --reas-group 11" $rep || exit 1
  one m_t512_g7 t512 "--mtu 9000 --reas-group 7" $rep || exit 1
  one m_t768 t768 "--mtu 9000" $rep || exit 1
  one m_t768_g11 t768 "--mtu 9000 --reas-group 11" $rep || exit 1
done
