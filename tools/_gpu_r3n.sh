set -e
O=gpurun_out/r3n; mkdir -p $O
timeout -k 10 200 python bench.py --landing spread --subs none --cpu-seconds 0 --cold-steps 0 > $O/spread.json 2> $O/spread.err
timeout -k 10 200 python bench.py --landing spread --subs none --cpu-seconds 0 --cold-steps 0 --spread-eager > $O/spread_eager.json 2> $O/spread_eager.err
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_capi_exports.py -x -q --timeout 200 --timeout-method thread -m "gpu or not gpu" > $O/pytest.log 2>&1
E2SAR_BENCH_BACKEND=gloo E2SAR_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --landing spread --events 256 --cpu-seconds 0 --cold-steps 0 > $O/n2_spread.json 2> $O/n2_spread.err
