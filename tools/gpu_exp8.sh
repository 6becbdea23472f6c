#!/bin/bash
mkdir -p gpurun_out/exp8
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/exp8/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/exp8/$name.log) $(grep -o '"simd_active_lanes[^}]*' gpurun_out/exp8/$name.log)"; return $rc; }
MTSG_TRACE_MODE=8 timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/exp8/pytest_m8.log 2>&1; rc=$?; tail -n 1 gpurun_out/exp8/pytest_m8.log; [ $rc -ne 0 ] && exit $rc
for m in 6 8 9 10 11; do
  MTSG_TRACE_MODE=$m run "m$m" 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
done
