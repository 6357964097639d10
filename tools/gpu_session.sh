#!/bin/bash
# One parametrised GPU session (replaces round 4's single-use tools/r4_gpu*.sh scripts).
# Every step runs under its own time limit; the session stops at the first failing step.
# Output goes to gpurun_out/$TAG/.
#
#   tools/gpu_session.sh TAG STEP [STEP...]
#     pytest[=FILES]        GPU suite (default: all of tests/ -m gpu), FILES comma-separated
#     ab=REPS:ARGS:NAMES    interleaved bench A/B of library builds (tools/ab_libs.sh);
#                           NAMES comma-separated, "base" = the tree's library
#     prof=WORKLOADS        rocprofv3 stats + PMC per workload (tools/profile_round4.sh)
#     bench=ARGS            one bench.py run, its JSON line to bench_N.json
#     smoke                 __graft_entry__.smoke()
#     cmd=SHELL             any other command (its own 300 s limit)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
n=0
for step in "$@"; do
  n=$((n + 1))
  key=${step%%=*}; val=${step#*=}; [ "$key" = "$step" ] && val=""
  echo "== step $n $key $(date +%T)" | tee -a $O/progress.log
  case $key in
    pytest)
      files=${val:-tests}; files=${files//,/ }
      timeout -k 10 900 python -u -m pytest $files -m gpu -x -q --timeout 120 --timeout-method thread \
        > $O/pytest_$n.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_$n.log; exit 1; }
      tail -2 $O/pytest_$n.log ;;
    ab)
      IFS=: read -r reps args names <<< "$val"
      tools/ab_libs.sh $TAG/ab_$n $reps "$args" ${names//,/ } || exit 1 ;;
    prof)
      tools/profile_round4.sh $O/prof_$n ${val//,/ } || { echo "profile failed"; tail -5 $O/prof_$n/*/*.log; exit 1; }
      for f in $O/prof_$n/*/pmc_summary.json; do python3 - $f <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    print(sys.argv[1].split("/")[-2], k, round((v["fetch_bytes_per_launch"] or 0) / 1e6, 1), "MB read",
          round((v["write_bytes_per_launch"] or 0) / 1e6, 1), "MB write")
PY
      done ;;
    bench)
      timeout -k 10 400 python bench.py $val > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench failed"; tail -20 $O/bench_$n.err; exit 1; }
      tail -c 600 $O/bench_$n.json; echo ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    cmd)
      timeout -k 10 300 bash -c "$val" > $O/cmd_$n.log 2>&1 || { echo "cmd failed"; tail -20 $O/cmd_$n.log; exit 1; }
      tail -20 $O/cmd_$n.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $TAG done"
