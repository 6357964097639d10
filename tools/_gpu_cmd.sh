mkdir -p gpurun_out/abn
for be in 72 80 88 96 104 112; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 30 --reas pipelined --batch-events $be > gpurun_out/abn/pipe_$be.json 2> gpurun_out/abn/pipe_$be.err || exit 1
done
for be in 112 128; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 30 --reas fused --batch-events $be > gpurun_out/abn/fused_$be.json 2> gpurun_out/abn/fused_$be.err || exit 1
done
