#!/bin/bash
# LDS-slab reassembly: copy microbenchmark, GPU suite on the slab library, A/B against the
# round-4 head (register-round reas_kernel); then the staged chunk-range scatter pass (r4_gpu11)
# (inside build/snap)
set -o pipefail
ROOTDIR=$(cd ../.. && pwd)
O=gpurun_out/r4_gpu12
mkdir -p $O
timeout -k 10 120 $ROOTDIR/build/ub/ubench_slab 15 > $O/ubench_slab.json 2> $O/ubench_slab.err || { echo "ubench failed"; cat $O/ubench_slab.err; exit 1; }
cat $O/ubench_slab.json
E2SAR_HIP_LIB=$ROOTDIR/build/variants/lib_slab.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_slab.log 2>&1 || { echo "pytest (slab) failed"; tail -60 $O/pytest_slab.log; exit 1; }
tail -2 $O/pytest_slab.log
ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu12/head 3 "" base slab > $O/head.log 2>&1 || { echo "head A/B failed"; cat $O/head.log; exit 1; }
cat $O/head.log
ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu12/m9k 2 "--mtu 9000" base slab > $O/m9k.log 2>&1 || { echo "m9k A/B failed"; cat $O/m9k.log; exit 1; }
cat $O/m9k.log
bash tools/r4_gpu11.sh
