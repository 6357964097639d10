set -e
O=gpurun_out/r3g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1
tools/ab_variants.sh r3g/ab "--subs none" base shift1 shift2 pre
timeout -k 10 200 python bench.py --landing spread --subs none --cpu-seconds 0 --cold-steps 0 > $O/spread.json 2> $O/spread.err
