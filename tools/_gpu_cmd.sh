set -e
O=gpurun_out/s2b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
tools/gpu_profile.sh s2prof
python tools/pmc_summary.py gpurun_out/s2prof/fetch gpurun_out/s2prof/write gpurun_out/s2prof/pmc_summary.json --workload mtu=1500,event_bytes=1048576,batch_events=128,lb_version=2 > /dev/null
cat gpurun_out/s2prof/bench.json
