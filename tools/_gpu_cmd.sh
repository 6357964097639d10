set -e
O=gpurun_out/chk3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline'])"
timeout -k 10 200 python tools/ub_concurrency.py > $O/conc.json; cat $O/conc.json
