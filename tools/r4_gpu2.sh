#!/bin/bash
# Round 4, pass 2 (inside build/snap): the experimental library's load check, an A/B of
# round-3 kernel knobs against the round-2 head, the two-rank spread rehearsal, then the
# evidence: default bench line, isolated per-workload profiles, config 3's two speeds.
set -o pipefail
O=gpurun_out/r4_gpu2
mkdir -p $O
ROOTDIR=$(cd ../.. && pwd)
timeout -k 10 120 python3 -c "
import torch; print('torch sees', torch.cuda.device_count(), torch.cuda.is_available())
import os; os.environ['E2SAR_HIP_LIB']=os.path.abspath('build/variants/lib_experimental.so')
from e2sar_amd import sar, _capi; print('lib', _capi.LIB_PATH, _capi.has_experimental())
c=sar.Context(0); print('ctx ok')
" > $O/exp_load.log 2>&1; echo "exp_load rc=$?" >> $O/exp_load.log
E2SAR_HIP_LIB=$(pwd)/build/variants/lib_experimental.so timeout -k 10 300 python -u -m pytest tests/test_gpu_chained.py tests/test_gpu_xcd_groups.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exp.log 2>&1; echo "exp rc=$?" >> $O/pytest_exp.log
E2SAR_BENCH_BACKEND=gloo E2SAR_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --cpu-seconds 0 --cold-steps 0 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { echo "n2 failed"; tail -30 $O/bench_n2_gloo.err; exit 1; }
for rep in 1 2; do
  (cd build/ab_r2 && timeout -k 10 200 python bench.py --cpu-seconds 0 --cold-steps 0 --quiet) > $O/r2_$rep.json 2>/dev/null
  ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu2/knobs 1 "" base nostripe edge0 nodefer >> $O/knobs.log 2>&1 || { echo "knobs failed"; tail $O/knobs.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/r2_$rep.json').read().strip().splitlines()[-1]); print('r2', d['value'], d['roofline']['avg_launch_ms'])" >> $O/knobs.log
done
cat $O/knobs.log
echo done
