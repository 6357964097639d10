set -e
O=gpurun_out/relay; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "relay or roundtrip" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for b in 32 64; do timeout -k 10 300 python tools/bench_hostpath.py --batch-events $b > $O/hp_b$b.json; cat $O/hp_b$b.json; done
timeout -k 10 300 python tools/bench_hostpath.py --batch-events 64 --mtu 9000 > $O/hp9_b64.json; cat $O/hp9_b64.json
