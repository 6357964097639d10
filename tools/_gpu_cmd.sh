set -e
A="--subs none --cold-steps 0 --cpu-seconds 0"
tools/ab_args.sh r3s3_gs2 "g4|$A" "g20|$A --graph-steps 20" "g4|$A" "g20|$A --graph-steps 20" "g4|$A" "g20|$A --graph-steps 20" "g4|$A" "g20|$A --graph-steps 20"
