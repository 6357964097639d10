mkdir -p gpurun_out/cfg3
tools/ab_variants.sh cfg3/a "--steps 30" base c4k c12k
tools/ab_variants.sh cfg3/b "--steps 30 --mtu 9000" base c4k c12k
tools/ab_variants.sh cfg3/c "--mtu 9000 --event-bytes 8388608 --events 280 --batch-events 16" base c4k c12k
tools/ab_variants.sh cfg3/d "--mtu 9000 --event-bytes 8388608 --events 280 --batch-events 8" base
tools/ab_variants.sh cfg3/e "--mtu 9000 --event-bytes 8388608 --events 280 --batch-events 32" base
