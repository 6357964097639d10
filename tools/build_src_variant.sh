#!/bin/bash
# A/B build of libe2sar_hip.so from an edited copy of the kernel sources (the product sources
# carry no build-time switches): copies e2sar_amd/csrc to build/variants/src_NAME, applies
# each sed expression to sar_kernels.hip, builds build/variants/lib_NAME.so.
#   tools/build_src_variant.sh NAME 'sed-expr' ['sed-expr'...]
set -e
N=$1; shift
D=build/variants/src_$N
rm -rf $D && mkdir -p $D && cp e2sar_amd/csrc/*.hip e2sar_amd/csrc/*.hpp e2sar_amd/csrc/*.cpp $D/
for e in "$@"; do sed -i -e "$e" $D/sar_kernels.hip; done
if cmp -s $D/sar_kernels.hip e2sar_amd/csrc/sar_kernels.hip; then echo "variant $N: no change"; exit 1; fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -I$D -shared \
  -o build/variants/lib_$N.so $D/sar_kernels.hip $D/capi.cpp
echo "built build/variants/lib_$N.so"
