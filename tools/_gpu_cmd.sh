set -e
O=gpurun_out/r3s3_contig2; mkdir -p $O
L=$GRAFT_REPO_ROOT/build/variants/lib_contig.so
E2SAR_HIP_LIB=$L timeout -k 10 300 python tools/place_probe.py --trials 2 --shifts-mib 0 --pk-lib \
  --offsets-mib 0,0.00390625,0.0078125,0.015625,0.03125,0.0625,0.125,0.25,0.5,1,1.5,2,3,4,6,8,12,16,24,32 > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
python -c "
import json
for l in open('$O/probe.jsonl'):
    d=json.loads(l); print(d['pk_off'], d['arena_rel'], d['seg_us'], d['reas_us'])"
