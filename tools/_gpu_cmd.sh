set -e
O=gpurun_out/rehearse4; mkdir -p $O
export E2SAR_BENCH_BACKEND=gloo E2SAR_BENCH_SHARE_GPU=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 5 --warmup 2 --events 256 > $O/own4.json 2> $O/own4.err || { tail -20 $O/own4.err; exit 1; }
python -c "import json;d=json.load(open('$O/own4.json'));print(d['n_gpus'],d['value'],d['config']['parallelism'],d['config']['verified_roundtrip'])"
