#!/bin/bash
# Round-3 evidence on one MI355X: for each workload, a rocprofv3 --kernel-trace --stats pass
# of bench.py and (headline, mtu9000, config3) the FETCH_SIZE and WRITE_SIZE PMC passes,
# summarised by tools/pmc_summary.py.  Usage: tools/profile_round3.sh OUTDIR [workload...]
# (workloads: headline mtu9000 config3 spread pre; default all)
set -e
R=$(pwd)
O=$R/$1; shift
mkdir -p $O
W=${@:-headline mtu9000 config3 spread pre}
cd /tmp && export TMPDIR=/tmp
for w in $W; do
  case $w in
    headline) A="--subs none"; WL="mtu=1500,event_bytes=1048576,batch_events=205,lb_version=2";;
    mtu9000)  A="--subs none --mtu 9000"; WL="mtu=9000,event_bytes=1048576,batch_events=205,lb_version=2";;
    config3)  A="--subs none --mtu 9000 --event-bytes 8388608 --events 280 --batch-events 70 --cold-batch-events 35"; WL="mtu=9000,event_bytes=8388608,batch_events=70,lb_version=2";;
    spread)   A="--subs none --landing spread --cold-steps 0"; WL="";;
    pre)      A="--subs none --cold-steps 0"; WL="";;
  esac
  if [ $w = pre ]; then export E2SAR_HIP_LIB=$R/build/variants/lib_pre.so; else unset E2SAR_HIP_LIB; fi
  mkdir -p $O/$w
  echo "== $w stats" >> $O/progress.log
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$w/stats -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 8 --warmup 1 --cold-steps 4 $A > $O/$w/bench_profiled.json 2> $O/$w/stats.log
  if [ -n "$WL" ]; then
    echo "== $w pmc" >> $O/progress.log
    timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/$w/fetch -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 2 --warmup 1 --cold-steps 2 --no-verify --eager $A > $O/$w/fetch.log 2>&1
    timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/$w/write -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 2 --warmup 1 --cold-steps 2 --no-verify --eager $A > $O/$w/write.log 2>&1
    python3 $R/tools/pmc_summary.py $O/$w/fetch $O/$w/write $O/$w/pmc_summary.json --workload $WL > /dev/null
  fi
done
echo done >> $O/progress.log
