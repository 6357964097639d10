#!/bin/bash
# per-variant rocprof stats of the reference-order bench
set -e
OUT=${OUT:-ro_ab}
R=$(pwd)
mkdir -p gpurun_out/$OUT
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-product}; do
  if [ $v = product ]; then L=""; else L=$R/build/variants/lib_$v.so; fi
  E2SAR_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$OUT/$v -o run -- python3 $R/bench.py --reference-order --subs none --cold-steps 0 --cpu-seconds 0 --steps 8 --no-verify > $R/gpurun_out/$OUT/$v.json 2> $R/gpurun_out/$OUT/$v.err
done
