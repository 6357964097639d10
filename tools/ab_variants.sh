#!/bin/bash
# Run bench.py once per variant library (build/variants/lib_<name>.so; "base" = in-tree lib).
# Usage: tools/ab_variants.sh TAG "bench args" name...
set -e
TAG=$1; ARGS=$2; shift 2
mkdir -p gpurun_out/$TAG
for v in "$@"; do
  if [ "$v" = base ]; then L=$GRAFT_REPO_ROOT/e2sar_amd/lib/libe2sar_hip.so; else L=$GRAFT_REPO_ROOT/build/variants/lib_$v.so; fi
  E2SAR_HIP_LIB=$L timeout -k 10 200 python bench.py --cpu-seconds 0 $ARGS > gpurun_out/$TAG/$v.json 2> gpurun_out/$TAG/$v.err
done
