#!/bin/bash
# Write / read request mix of one bench workload per library build (round 5, config 3's XCD
# order): TCC_EA0_WRREQ (all write requests) against TCC_EA0_WRREQ_64B (whole 64-byte
# requests), TCC_EA0_RDREQ and TCC_EA0_RDREQ_DRAM, one PMC pass per library.
# Usage: tools/pmc_wrreq.sh OUTDIR "bench args" name...   ("base" = the tree's library)
R=$(pwd)
O=$R/$1; ARGS=$2; shift 2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then L=$R/e2sar_amd/lib/libe2sar_hip.so; else L=$R/build/variants/lib_$v.so; fi
  E2SAR_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-trace --output-format csv -d $O/$v -o run -- python3 $R/bench.py --cpu-seconds 0 --subs none --cold-steps 0 --steps 2 --warmup 1 --no-verify --eager $ARGS > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  python3 - $O/$v <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for r in rows:
    k = r.get("Kernel_Name", "")[:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
for k, c in agg.items():
    n = max(1, len(cnt[k]))
    if c.get("TCC_EA0_WRREQ_sum", 0) / n < 1e5: continue
    print(sys.argv[1].split("/")[-1], k, {kk: round(v / n) for kk, v in sorted(c.items())})
PY
done
