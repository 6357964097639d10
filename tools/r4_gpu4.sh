#!/bin/bash
# Round 4, pass (inside build/snap): fused-kernel variants against the default build,
# the datagram-shape microbenchmark, a bisect of round 3's kernel commits (each tree with
# its own bench), the A/B-only forms against their library.
set -o pipefail
O=gpurun_out/r4_gpu4
mkdir -p $O
ROOTDIR=$(cd ../.. && pwd)
timeout -k 10 150 $ROOTDIR/build/ubench_rounds 210 11 > $O/ubench_rounds.json 2> $O/ubench_rounds.err || { echo "ubench failed"; cat $O/ubench_rounds.err; exit 1; }
cat $O/ubench_rounds.json
ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu4/var 2 "" base g16 g16c g24 rf > $O/var.log 2>&1 || { echo "var failed"; tail $O/var.log; exit 1; }
cat $O/var.log
for c in r2 bis_d55a3df bis_c82406f bis_d1d1d1c bis_7f29271 bis_6203807; do
  if [ $c = r2 ]; then d=$ROOTDIR/build/ab_r2; else d=$ROOTDIR/build/$c; fi
  S=""; grep -q -- '"--subs"' $d/bench.py && S="--subs none"
  (cd $d && timeout -k 10 200 python bench.py --cpu-seconds 0 --cold-steps 0 $S --quiet) > $O/bis_$c.json 2> $O/bis_$c.err || { echo "$c failed"; tail -5 $O/bis_$c.err; continue; }
  python3 -c "
import json; d=json.loads(open('$O/bis_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['roofline']['avg_launch_ms'])"
done > $O/bisect.log 2>&1
(cd . && timeout -k 10 200 python bench.py --cpu-seconds 0 --cold-steps 0 --subs none --quiet) > $O/bis_head.json 2>/dev/null && python3 -c "
import json; d=json.loads(open('$O/bis_head.json').read().strip().splitlines()[-1]); print('head', d['value'], d['roofline']['avg_launch_ms'])" >> $O/bisect.log
cat $O/bisect.log
E2SAR_HIP_LIB=$(pwd)/build/variants/lib_experimental.so timeout -k 10 300 python -u -m pytest tests/test_gpu_chained.py tests/test_gpu_xcd_groups.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exp.log 2>&1; echo "exp rc=$?"; tail -2 $O/pytest_exp.log
echo done
