set -e
O=gpurun_out/r3o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest.log 2>&1
E2SAR_BENCH_BACKEND=gloo E2SAR_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --landing spread --events 256 --cpu-seconds 0 --cold-steps 0 > $O/n2_spread.json 2> $O/n2_spread.err
