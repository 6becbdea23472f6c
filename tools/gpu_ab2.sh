#!/bin/bash
# A/B of two device libraries on one box: bench lines alternating.
#   tools/gpu_ab2.sh <libA relative path|cur> <libB> [bench args...]
O=gpurun_out/ab; mkdir -p $O
A=$1; B=$2; shift 2
for rep in 1 2; do
  for L in $A $B; do
    if [ "$L" = cur ]; then unset MTSG_LIB; else export MTSG_LIB=$L; fi
    timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-parity "$@" > $O/run.log 2>&1 || { tail $O/run.log; exit 1; }
    echo "$L rep$rep: $(python tools/summarize_bench.py $O/run.log)"
  done
done
