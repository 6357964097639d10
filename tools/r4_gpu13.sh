#!/bin/bash
# fused reassembly workgroup size A/B: 256 (base) vs 384 / 512 / 1024 threads, at the
# balanced group size and at group sizes of whole copy rounds (repository root)
set -o pipefail
O=gpurun_out/r4_gpu13
mkdir -p $O
run() {  # tag reps "args" libs...
  local t=$1 r=$2 a=$3; shift 3
  tools/ab_libs.sh r4_gpu13/$t $r "$a" "$@" > $O/$t.log 2>&1 || { echo "$t failed"; cat $O/$t.log; exit 1; }
  echo "== $t ($a)"; cat $O/$t.log
}
run head 3 "" base t384 t512 t1024
run g44 2 "--reas-group 44" base t512
run g33 2 "--reas-group 33" base t384
run m9k 2 "--mtu 9000" base t384 t512
