set -e
O=gpurun_out/r3host; mkdir -p $O
for c in dma kernel-d2h kernel; do
  timeout -k 10 200 python tools/bench_hostpath.py --batch-events 64 --copy $c > $O/$c.json 2> $O/$c.err
done
