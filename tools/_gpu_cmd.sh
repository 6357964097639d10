mkdir -p gpurun_out/n2
export E2SAR_BENCH_BACKEND=gloo E2SAR_BENCH_SHARE_GPU=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --cpu-seconds 0 --events 256 > gpurun_out/n2/own.json 2> gpurun_out/n2/own.err || { tail -20 gpurun_out/n2/own.err; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --steps 10 --warmup 2 --cpu-seconds 0 --events 128 > gpurun_out/n2/own4.json 2> gpurun_out/n2/own4.err || { tail -20 gpurun_out/n2/own4.err; exit 1; }
