mkdir -p gpurun_out/abr
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/abr/tests.log 2>&1 || { tail -30 gpurun_out/abr/tests.log; exit 1; }
tail -2 gpurun_out/abr/tests.log
for m in fused split; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --reas $m > gpurun_out/abr/$m.json 2> gpurun_out/abr/$m.err || exit 1
done
timeout -k 10 200 python bench.py --cpu-seconds 0 --reas fused --batch-events 64 > gpurun_out/abr/fused64.json 2> gpurun_out/abr/fused64.err
