#!/bin/bash
# destination-aligned / LDS-staged scatter stores on config 3 (inside build/snap)
set -o pipefail
O=gpurun_out/r4_gpu8
mkdir -p $O
ROOTDIR=$(cd ../.. && pwd)
ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu8/c3 2 "--mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70" base sh1 sh2 sh3 > $O/c3.log 2>&1 || { echo "c3 failed"; cat $O/c3.log; exit 1; }
cat $O/c3.log
ROOTDIR=$ROOTDIR tools/ab_libs.sh r4_gpu8/hq 2 "" base hq1536 hq768 hqall > $O/hq.log 2>&1 || { echo "hq failed"; cat $O/hq.log; exit 1; }
cat $O/hq.log
