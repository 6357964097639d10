O=gpurun_out/r3i; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 ./build/e2sar_perf --loopback -l 1048576 -n 2000 -m 9000 --rate -1 --sockets 4 --port 10600 > $O/lo_9000_s4_r$r.log 2>&1
  grep -E "End-to-end|Completed|Received" $O/lo_9000_s4_r$r.log
done
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
