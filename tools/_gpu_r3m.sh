set -e
O=gpurun_out/r3m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_large_batch.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest.log 2>&1
tools/ab_variants.sh r3m/a "--subs none --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70 --cold-steps 0" base parts1 parts3 parts4
tools/ab_variants.sh r3m/b "--subs none --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70 --cold-steps 0" base parts1 parts3 parts4
