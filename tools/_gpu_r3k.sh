set -e
O=gpurun_out/r3k; mkdir -p $O
E2SAR_BENCH_BACKEND=gloo E2SAR_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --cpu-seconds 0 --cold-steps 0 > $O/n2_own.json 2> $O/n2_own.err
E2SAR_BENCH_BACKEND=gloo E2SAR_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --landing spread --events 256 --cpu-seconds 0 --cold-steps 0 > $O/n2_spread.json 2> $O/n2_spread.err
