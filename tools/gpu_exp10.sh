#!/bin/bash
mkdir -p gpurun_out/exp10
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/exp10/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/exp10/$name.log) $(grep -o '"nodes_per_ray[^}]*' gpurun_out/exp10/$name.log | cut -c1-200)"; return $rc; }
MTSG_TRACE_MODE=12 timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/exp10/pytest_m12.log 2>&1; rc=$?; tail -n 1 gpurun_out/exp10/pytest_m12.log; [ $rc -ne 0 ] && exit $rc
for m in 6 12 13; do
  MTSG_TRACE_MODE=$m run "m$m" 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
done
MTSG_TRACE_MODE=12 run "m12_cbox" 300 python bench.py --steps 2 --warmup 1 --no-cpu --workload cbox || exit $?
