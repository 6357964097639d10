#!/bin/bash
# The façade over UDP loopback (build/e2sar_perf --loopback: Segmenter -> sockets ->
# Reassembler, unpaced): 2000 x 1 MiB events at MTU 1500 and 9000, 1 and 4 send sockets.
# Usage: tools/facade_loopback.sh TAG
set -e
O=gpurun_out/$1; mkdir -p $O
for m in 1500 9000; do
  for s in 1 4; do
    timeout -k 10 200 ./build/e2sar_perf --loopback -l 1048576 -n 2000 -m $m --rate -1 --sockets $s --port 10600 \
      > $O/lo_${m}_s$s.log 2>&1 || { tail -20 $O/lo_${m}_s$s.log; exit 1; }
    grep -E "End-to-end|Received" $O/lo_${m}_s$s.log
  done
done
