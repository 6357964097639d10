#!/bin/bash
# One rocprofv3 --pmc pass per library build over one bench workload, counters summed over
# the chip and averaged per launch of each kernel (round 5).  At most 4 TCC counters a pass.
# Usage: tools/pmc_pass.sh OUTDIR "COUNTER COUNTER ..." "bench args" name...
#        ("base" = the tree's library, NAME = build/variants/lib_NAME.so)
R=$(pwd)
O=$R/$1; CNT=$2; ARGS=$3; shift 3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then L=$R/e2sar_amd/lib/libe2sar_hip.so; else L=$R/build/variants/lib_$v.so; fi
  E2SAR_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $O/$v -o run -- python3 $R/bench.py --cpu-seconds 0 --subs none --cold-steps 0 --steps 2 --warmup 1 --no-verify --eager $ARGS > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  python3 - $O/$v <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for r in rows:
    k = r.get("Kernel_Name", "")[:70]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
for k, c in agg.items():
    n = max(1, len(cnt[k]))
    if "e2sar" not in k: continue
    print(sys.argv[1].split("/")[-1], k, n, "launches", {kk: round(v / n) for kk, v in sorted(c.items())})
PY
done
