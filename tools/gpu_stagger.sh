#!/bin/bash
# Staggered lanes (MTSG_LANES / MTSG_STAGGER) at the emulated 8-rank share and the whole frame
O=gpurun_out/stagger; mkdir -p $O
run() { local tag=$1 e=$2 l=$3 g=$4; MTSG_LANES=$l MTSG_STAGGER=$g timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --emulate-ranks $e > $O/$tag.log 2>&1 || exit $?; echo "$tag $(python tools/summarize_bench.py $O/$tag.log)"; }
for cfg in ${CFGS:-"8 1 0" "8 2 0" "8 2 2" "8 2 3" "8 3 2" "8 4 2" "1 1 0" "1 2 3"}; do
  set -- $cfg; run e$1_l$2_s$3 $1 $2 $3
done
