set -e
O=gpurun_out/ent; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dataplane_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
