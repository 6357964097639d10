#!/bin/bash
# smoke + N=2 rehearsal (gloo, both ranks on GPU 0) on the 768/512-thread kernel, then
# config 3's two speeds: buffer x arena reallocation probe in two processes (repository root)
set -o pipefail
O=gpurun_out/r4_gpu18
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
E2SAR_BENCH_BACKEND=gloo E2SAR_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --cpu-seconds 0 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { echo "n2 failed"; tail -30 $O/bench_n2_gloo.err; exit 1; }
tail -c 400 $O/bench_n2_gloo.json; echo
for p in 1 2; do
  timeout -k 10 300 python tools/realloc_probe.py > $O/realloc_p$p.jsonl 2> $O/realloc_p$p.err || { echo "probe failed"; tail -20 $O/realloc_p$p.err; exit 1; }
  tail -1 $O/realloc_p$p.jsonl
done
