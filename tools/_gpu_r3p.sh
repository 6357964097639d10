set -e
O=gpurun_out/r3p; mkdir -p $O
tools/ab_variants.sh r3p/a "--subs none" base ntst0 fntst0
tools/ab_variants.sh r3p/b "--subs none" base ntst0 fntst0
