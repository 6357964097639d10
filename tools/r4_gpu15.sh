#!/bin/bash
# 768/512-thread fused reassembly as the default: GPU suite, A/B against 256 threads, group
# sizes at 768, then the round's evidence pass (default bench line, per-workload rocprof +
# PMC) (repository root)
set -o pipefail
O=gpurun_out/r4_gpu15
mkdir -p $O
E2SAR_RANDOM_SEEDS=40 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
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
  one h_t256 t256 "" $rep || exit 1
  one h_g49 base "--reas-group 49" $rep || exit 1
  one h_g64 base "--reas-group 64" $rep || exit 1
  one m_base base "--mtu 9000" $rep || exit 1
  one m_t256 t256 "--mtu 9000" $rep || exit 1
done
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
tail -c 600 $O/bench_default.json
timeout -k 10 1500 tools/profile_round4.sh $O/prof || { echo "profile failed"; cat $O/prof/progress.log; exit 1; }
cat $O/prof/progress.log
bash tools/r4_gpu16.sh
