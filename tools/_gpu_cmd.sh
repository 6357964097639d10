mkdir -p gpurun_out/fin1
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/fin1/tests.log 2>&1 || { tail -30 gpurun_out/fin1/tests.log; exit 1; }
tail -2 gpurun_out/fin1/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin1/smoke.log 2>&1 || { tail -20 gpurun_out/fin1/smoke.log; exit 1; }
timeout -k 10 300 python tools/bench_hostpath.py > gpurun_out/fin1/hostpath.json 2> gpurun_out/fin1/hostpath.err || exit 1
timeout -k 10 300 python tools/bench_hostpath.py --batch-events 64 > gpurun_out/fin1/hostpath64.json 2>> gpurun_out/fin1/hostpath.err || exit 1
tools/gpu_profile.sh fin1/prof
