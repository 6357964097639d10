set -e
E2SAR_HIP_LIB=$GRAFT_REPO_ROOT/build/variants/lib_trace.so timeout -k 10 200 python tools/trace_reas.py > gpurun_out/tr_seg.json
python -c "
import json;d=json.load(open('gpurun_out/tr_seg.json'))['seg'];print({k:v for k,v in d.items() if k!='running_per_2us'});print(d['running_per_2us'])"
