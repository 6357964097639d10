set -e
O=gpurun_out/perf_tool; mkdir -p $O
for m in 9000 1500; do timeout -k 10 200 ./build/e2sar_perf --loopback -l 1048576 -n 2000 -m $m --rate -1 --port 10600 > $O/m$m.txt 2>&1 || { tail -20 $O/m$m.txt; exit 1; }; tail -6 $O/m$m.txt; done
