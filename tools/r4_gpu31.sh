#!/bin/bash
# jumbo fused kernel at 2 workgroups per CU (j2) and the cold scatter cap at 7 per CU (c7)
# vs the defaults, and the config-3 profile on the seg_kernel<4> cap (repository root)
set -o pipefail
O=gpurun_out/r4_gpu31
mkdir -p $O
tools/ab_libs.sh r4_gpu31/m 3 "--mtu 9000" base j2 > $O/m.log 2>&1 || { echo "m failed"; cat $O/m.log; exit 1; }
cat $O/m.log
tools/ab_libs.sh r4_gpu31/cold 2 "--cold-steps 10" base c7 > $O/cold.log 2>&1 || { echo "cold failed"; cat $O/cold.log; exit 1; }
for f in $O/cold/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d.get('reas_cold')
print('  cold', '$f'.split('/')[-1], c['value'], c['roofline']['avg_launch_ms'], c['roofline']['frac']) if c else None"; done
timeout -k 10 600 tools/profile_round4.sh $O/prof config3 || { echo "profile failed"; cat $O/prof/progress.log; exit 1; }
cat $O/prof/progress.log
