set -e
O=gpurun_out/r3j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_large_batch.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1
tools/ab_variants.sh r3j/c3 "--subs none --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70 --cold-steps 0" base norev base norev
tools/ab_variants.sh r3j/hl "--subs none --cold-steps 0" base frev base frev
