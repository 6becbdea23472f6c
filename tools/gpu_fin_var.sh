#!/bin/bash
# tail kernel: shading batch size (MTSG_FINISH_SHADE_MIN) x threshold at the emulated 8-rank share
O=gpurun_out/ab; mkdir -p $O
for L in cur abtest/libmtsg_fw4.so; do
  if [ "$L" = cur ]; then unset MTSG_LIB; else export MTSG_LIB=$L; fi
  for m in 8 24 48; do
  for f in 524288 1048576; do
    MTSG_FINISH_SHADE_MIN=$m MTSG_FINISH=$f timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu --no-parity --emulate-ranks 8 > $O/e8.log 2>&1 || { tail $O/e8.log; exit 1; }
    echo "$L m=$m fin=$f $(python tools/summarize_bench.py $O/e8.log)"
  done
  done
done
