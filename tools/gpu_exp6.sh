#!/bin/bash
# unified traversal (modes 5-7) vs while-while (mode 3); short-stack sizes
mkdir -p gpurun_out/exp6
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/exp6/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/exp6/$name.log) $(grep -o '"simd_active_lanes[^}]*' gpurun_out/exp6/$name.log)"; return $rc; }
for m in 5; do
  MTSG_TRACE_MODE=$m timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/exp6/pytest_m$m.log 2>&1; rc=$?; tail -n 1 gpurun_out/exp6/pytest_m$m.log; [ $rc -ne 0 ] && exit $rc
done
for m in 3 5 6 7; do
  MTSG_TRACE_MODE=$m run "m$m" 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
done
for v in s6 s4 s12; do
  MTSG_LIB=build/var/libmtsg_$v.so MTSG_TRACE_MODE=5 run "m5_$v" 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
done
MTSG_TRACE_MODE=5 run m5_cbox 300 python bench.py --steps 2 --warmup 1 --no-cpu --workload cbox || exit $?
