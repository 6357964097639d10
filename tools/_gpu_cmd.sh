mkdir -p gpurun_out/perf2
timeout -k 10 300 python -m pytest tests/test_dataplane_gpu.py -x -q > gpurun_out/perf2/tests.log 2>&1 || { tail -30 gpurun_out/perf2/tests.log; exit 1; }
tail -1 gpurun_out/perf2/tests.log
for r in 5 10 20; do
timeout -k 10 120 ./build/e2sar_perf --loopback -l 1048576 -n 2000 -m 9000 --rate $r > gpurun_out/perf2/lo_9000_r$r.log 2>&1; echo "rc=$?" >> gpurun_out/perf2/lo_9000_r$r.log
done
timeout -k 10 120 ./build/e2sar_perf --loopback -l 1048576 -n 2000 -m 1500 --rate 5 > gpurun_out/perf2/lo_1500_r5.log 2>&1; echo "rc=$?" >> gpurun_out/perf2/lo_1500_r5.log
