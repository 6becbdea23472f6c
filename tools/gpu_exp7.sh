#!/bin/bash
mkdir -p gpurun_out/exp7
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/exp7/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/exp7/$name.log) $(grep -o '"simd_active_lanes[^}]*' gpurun_out/exp7/$name.log)"; return $rc; }
for v in s6 s5 s6f128 s6f512; do
  for m in 5 6 7; do
    MTSG_LIB=build/var/libmtsg_$v.so MTSG_TRACE_MODE=$m run "${v}_m$m" 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
  done
done
