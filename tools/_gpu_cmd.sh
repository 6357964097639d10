set -e
O=gpurun_out/r3s3_dg3; mkdir -p $O
for a in "560 8976 8936" "560 1472 1436"; do
  timeout -k 10 200 ./build/ubench_dgram $a 10 | tee -a $O/dg.jsonl
done
