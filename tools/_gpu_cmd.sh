set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_flat.log 2>&1 || { tail -30 gpurun_out/pytest_flat.log; exit 1; }
tail -1 gpurun_out/pytest_flat.log
tools/ab_variants.sh r3s3_flat "--subs none --cold-steps 0" base flat0
cp gpurun_out/r3s3_flat/base.json gpurun_out/r3s3_flat/base1.json; cp gpurun_out/r3s3_flat/flat0.json gpurun_out/r3s3_flat/flat01.json
tools/ab_variants.sh r3s3_flat "--subs none --cold-steps 0" base flat0
O=$R/gpurun_out/r3s3_flat; cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --cpu-seconds 0 --steps 2 --warmup 1 --cold-steps 0 --no-verify --eager --subs none"
for v in base flat0; do
  if [ $v = base ]; then L=$R/e2sar_amd/lib/libe2sar_hip.so; else L=$R/build/variants/lib_$v.so; fi
  E2SAR_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAVES --kernel-trace --output-format csv -d $O/pmc_$v -o run -- python3 $B > $O/pmc_$v.log 2>&1
done
cd $R
for f in gpurun_out/r3s3_flat/*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['roofline']['avg_launch_ms'])"; done
