#!/bin/bash
# One GPU session of round evidence for a bench workload:
#   bench JSON, rocprofv3 kernel-trace stats (hot round trip + the cold receive leg),
#   FETCH_SIZE and WRITE_SIZE PMC passes (separate runs, no tracing domains besides kernels).
# Usage: tools/gpu_profile.sh TAG [extra bench args...]
set -e
TAG=$1; shift
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python bench.py "$@" > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 10 --warmup 1 --cold-steps 8 "$@" > $O/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 3 --warmup 1 --cold-steps 2 --no-verify --eager "$@" > $O/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 3 --warmup 1 --cold-steps 2 --no-verify --eager "$@" > $O/write.log 2>&1
cd $R
find $O -name "*.csv" | head -20
