set -e
O=gpurun_out/oddskip; mkdir -p $O
E2SAR_REAS_ODD_SKIP=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest4.log 2>&1 || { tail -40 $O/pytest4.log; exit 1; }
tail -1 $O/pytest4.log
for r in 1 2; do for k in 0 8 5 4 3; do E2SAR_REAS_ODD_SKIP=$k timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 20 > $O/k${k}_$r.json; python -c "import json;d=json.load(open('$O/k${k}_$r.json'));print('skip $k',d['value'],d['roofline']['avg_launch_ms'])"; done; done
