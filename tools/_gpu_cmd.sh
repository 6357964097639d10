mkdir -p gpurun_out/hp2
timeout -k 10 300 python tools/bench_hostpath.py --batch-events 64 > gpurun_out/hp2/hostpath64.json 2> gpurun_out/hp2/err || exit 1
timeout -k 10 300 python tools/bench_hostpath.py --batch-events 32 > gpurun_out/hp2/hostpath32.json 2>> gpurun_out/hp2/err || exit 1
timeout -k 10 300 python tools/bench_hostpath.py --batch-events 64 --mtu 9000 > gpurun_out/hp2/hostpath64_9000.json 2>> gpurun_out/hp2/err || exit 1
