#!/bin/bash
# Round-4 evidence on one MI355X: every workload in a process of its own, so each kernel's
# rocprof average and PMC traffic belong to that workload alone (round 3's config-3 figures
# mixed in the cold leg's launches of the same kernel).  Per workload: a rocprofv3
# --kernel-trace --stats pass of bench.py, then separate FETCH_SIZE and WRITE_SIZE PMC
# passes, summarised by tools/pmc_summary.py.
# Usage: tools/profile_round4.sh OUTDIR [workload...]   (headline cold mtu9000 config3; default all)
set -e
R=$(pwd)
O=$R/$1; shift
mkdir -p $O
W=${@:-headline cold mtu9000 config3}
cd /tmp && export TMPDIR=/tmp
for w in $W; do
  case $w in
    headline) A="--subs none --cold-steps 0"; P="$A"; WL="mtu=1500,event_bytes=1048576,batch_events=205,lb_version=2";;
    cold)     A="--subs none --cold-steps 8"; P="--subs none --cold-steps 2"; WL="mtu=1500,event_bytes=1048576,batch_events=1024,lb_version=2";;
    mtu9000)  A="--subs none --cold-steps 0 --mtu 9000"; P="$A"; WL="mtu=9000,event_bytes=1048576,batch_events=205,lb_version=2";;
    config3)  A="--subs none --cold-steps 0 --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70"; P="$A"; WL="mtu=9000,event_bytes=8388608,batch_events=70,lb_version=2";;
  esac
  mkdir -p $O/$w
  echo "== $w stats $(date +%T)" >> $O/progress.log
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$w/stats -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 8 --warmup 1 $A > $O/$w/bench_profiled.json 2> $O/$w/stats.log
  # the same workload launched eagerly (no graph): rocprof's per-dispatch overhead inflates
  # the intervals of graph-replayed kernels, so kernel durations come from here
  echo "== $w eager stats $(date +%T)" >> $O/progress.log
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$w/stats_eager -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 8 --warmup 1 --eager $A > $O/$w/bench_profiled_eager.json 2> $O/$w/stats_eager.log
  echo "== $w pmc $(date +%T)" >> $O/progress.log
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/$w/fetch -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 2 --warmup 1 --no-verify --eager $P > $O/$w/fetch.log 2>&1
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/$w/write -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 2 --warmup 1 --no-verify --eager $P > $O/$w/write.log 2>&1
  python3 $R/tools/pmc_summary.py $O/$w/fetch $O/$w/write $O/$w/pmc_summary.json --workload $WL > /dev/null
done
echo done >> $O/progress.log
