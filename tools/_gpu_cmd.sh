set -e
tools/gpu_profile.sh s2prof205
python tools/pmc_summary.py gpurun_out/s2prof205/fetch gpurun_out/s2prof205/write gpurun_out/s2prof205/pmc_summary.json --workload mtu=1500,event_bytes=1048576,batch_events=205,lb_version=2 > /dev/null
cat gpurun_out/s2prof205/bench.json
