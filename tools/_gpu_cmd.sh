set -e
O=gpurun_out/r3s3_local; mkdir -p $O
for m in 221 64 1024; do timeout -k 10 120 ./build/ubench_local $m 10 | tee -a $O/local.jsonl; done
