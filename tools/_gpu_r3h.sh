set -e
O=gpurun_out/r3h; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1
tools/facade_loopback.sh r3h/facade > $O/facade.txt 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
