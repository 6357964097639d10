#!/bin/bash
# Build A/B variants of libe2sar_hip.so into build/variants/ (selected at run time with
# E2SAR_HIP_LIB=...).  Usage: tools/build_variants.sh name "-DFLAG=..." [name "-D..."]...
set -e
mkdir -p build/variants
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Ie2sar_amd/csrc -shared"
S="e2sar_amd/csrc/sar_kernels.hip e2sar_amd/csrc/capi.cpp"
while [ $# -gt 1 ]; do
  $H $2 -o build/variants/lib_$1.so $S &
  shift 2
done
wait
