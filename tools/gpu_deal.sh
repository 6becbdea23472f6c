#!/bin/bash
# Tile-deal row rotation (MTSG_DEAL_SKEW, measurement knob) on the emulated
# eight 1/8 C3 shares: per-share ms and the slowest share's speedup.
#   tools/gpu_deal.sh 1 0 3 ...
O=gpurun_out/deal; mkdir -p $O
export TMPDIR=/tmp
for k in "$@"; do
  MTSG_DEAL_SKEW=$k timeout -k 10 200 python bench.py --steps 10 --warmup 3 --emulate-ranks 8 --no-cpu --no-parity --no-count > $O/e8_skew$k.log 2>&1; rc=$?
  echo "skew $k rc=$rc $(grep -o '"share_speedup_min": [0-9.]*' $O/e8_skew$k.log) $(grep -o '"share_ms_per_step": \[[^]]*\]' $O/e8_skew$k.log)"
  if [ $rc -ne 0 ]; then tail -3 $O/e8_skew$k.log; exit $rc; fi
done
