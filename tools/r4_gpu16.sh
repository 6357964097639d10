#!/bin/bash
# scatter workgroup size A/B: 256 (base) vs 512 threads (s512: 16 datagrams @ 1500, 2 @ 9000;
# s512g3: 3 datagrams per workgroup) on config 3, the cold legs and the hot split form (repository root)
set -o pipefail
O=gpurun_out/r4_gpu16
mkdir -p $O
run() {  # tag "args" libs...
  local t=$1 a=$2; shift 2
  tools/ab_libs.sh r4_gpu16/$t 2 "$a" "$@" > $O/$t.log 2>&1 || { echo "$t failed"; cat $O/$t.log; exit 1; }
  echo "== $t ($a)"; cat $O/$t.log
  for f in $O/$t/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d.get('reas_cold')
print('  cold', '$f'.split('/')[-1], c['value'], c['roofline']['avg_launch_ms'], c['roofline']['frac']) if c else None"; done
}
run c3 "--mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70" base s512 s512g3
run cold9000 "--mtu 9000 --cold-steps 10" base s512 s512g3
run cold1500 "--cold-steps 10" base s512
run split "--reas split" base s512
run stripe "" base stripe0
run stripe9k "--mtu 9000" base stripe0
