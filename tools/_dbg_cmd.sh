mkdir -p gpurun_out/r3e
for v in base nopre noshift; do
  if [ "$v" = base ]; then L=$GRAFT_REPO_ROOT/e2sar_amd/lib/libe2sar_hip.so; else L=$GRAFT_REPO_ROOT/build/variants/lib_$v.so; fi
  E2SAR_HIP_LIB=$L timeout -k 10 100 python -u tools/debug_ro_graph.py > gpurun_out/r3e/$v.log 2>&1 || exit 1
done
