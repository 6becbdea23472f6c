#!/bin/bash
mkdir -p gpurun_out/exp13
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/exp13/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/exp13/$name.log) $(grep -o '"simd_active_lanes[^}]*' gpurun_out/exp13/$name.log)"; return $rc; }
MTSG_TRACE_MODE=14 timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/exp13/pytest_m14.log 2>&1; rc=$?; tail -n 3 gpurun_out/exp13/pytest_m14.log; [ $rc -ne 0 ] && exit $rc
for m in 12 14 15; do
  MTSG_TRACE_MODE=$m run "m$m" 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
done
for v in w7 s5; do
  MTSG_LIB=build/var/libmtsg_$v.so MTSG_TRACE_MODE=14 run "m14_$v" 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
done
MTSG_TRACE_MODE=14 run "m14_c5" 400 python bench.py --workload c5 --width 1920 --height 1080 --spp 64 --steps 2 --warmup 1 --no-cpu || exit $?
