#!/bin/bash
# A/B of events per launch (and 2-stream overlap) for the default workload; one JSON per run.
set -e
for be in 16 32 64 128 256; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 20 --batch-events $be > gpurun_out/ab_be$be.json 2>/dev/null
  timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 20 --batch-events $be --overlap > gpurun_out/ab_be${be}_ov.json 2>/dev/null
done
