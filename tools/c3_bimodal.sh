#!/bin/bash
# Config 3's two speeds: N config-3 bench processes back to back on one box,
# each under rocprofv3 --kernel-trace (per-launch durations), with the GPU's clocks, power
# and temperature sampled by rocm-smi every half second throughout, so a slow process can be
# matched against what the chip was doing.  Usage: tools/c3_bimodal.sh OUTDIR [N]
R=$(pwd)
O=$R/$1; N=${2:-6}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
( while true; do
    echo "T $(date +%s.%N)"
    rocm-smi --showclocks --showpower --showtemp --csv 2>/dev/null
    sleep 0.5
  done ) > $O/smi.log &
SMI=$!
trap "kill $SMI 2>/dev/null" EXIT
for i in $(seq 1 $N); do
  echo "P $i start $(date +%s.%N)" >> $O/marks.log
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/bench.py --cpu-seconds 0 --subs none --cold-steps 0 --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70 > $O/p$i.json 2> $O/p$i.err || { echo "process $i failed"; tail -5 $O/p$i.err; exit 1; }
  echo "P $i end $(date +%s.%N)" >> $O/marks.log
done
echo done
