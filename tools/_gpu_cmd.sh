set -e
O=gpurun_out/route2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_dist_gloo.py -x -q --timeout 120 --timeout-method thread -k "route or gloo or dist" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench.py --cpu-seconds 0 --landing spread > $O/spread.json
python -c "import json;d=json.load(open('$O/spread.json'));print('spread',d['value'],d['roofline']['avg_launch_ms'])"
