#!/bin/bash
# experimental-library GPU tests on the final kernels; fused group sizes around the balanced
# 59 at 768 threads (repository root)
set -o pipefail
O=gpurun_out/r4_gpu24
mkdir -p $O
E2SAR_HIP_LIB=$(pwd)/build/variants/lib_experimental.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_experimental.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_experimental.log; exit 1; }
tail -2 $O/pytest_experimental.log
one() {  # name "args" rep
  timeout -k 10 200 python bench.py --cpu-seconds 0 --cold-steps 0 --subs none $2 > $O/$1_$3.json 2> $O/$1_$3.err || { echo "$1 failed"; tail -5 $O/$1_$3.err; exit 1; }
  python3 - $O/$1_$3.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1].split("/")[-1], d["value"], r["avg_launch_ms"], r["frac"], flush=True)
PY
}
for rep in 1 2 3; do
  for g in 0 54 56 61; do one g$g "--reas-group $g" $rep || exit 1; done
done
