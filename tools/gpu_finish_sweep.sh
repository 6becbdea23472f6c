#!/bin/bash
# Tail-kernel switch point (MTSG_FINISH, paths) on the whole C3 frame and on
# the emulated 8-rank shares:  tools/gpu_finish_sweep.sh 262144 524288 ...
O=gpurun_out/fin3; mkdir -p $O
export TMPDIR=/tmp
for f in "$@"; do
  export MTSG_FINISH=$f
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 --no-cpu --no-parity --no-count > $O/e8_$f.log 2>&1; rc=$?
  echo "finish $f e8 rc=$rc $(grep -o '"value": [0-9.]*' $O/e8_$f.log) $(grep -o '"share_ms_per_step": \[[0-9., ]*\]' $O/e8_$f.log) $(grep -o '"whole_frame_ms_per_step": [0-9.]*' $O/e8_$f.log) $(grep -o '"share_speedup_min": [0-9.]*' $O/e8_$f.log)"
  if [ $rc -ne 0 ]; then tail -3 $O/e8_$f.log; exit $rc; fi
done
