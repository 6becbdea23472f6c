#!/bin/bash
# compact-state speculative traversal (modes 16/17) vs two-level (12) and speculative (14)
mkdir -p gpurun_out/exp14
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/exp14/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/exp14/$name.log)"; return $rc; }
MTSG_TRACE_MODE=16 timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/exp14/pytest_m16.log 2>&1; rc=$?; tail -n 3 gpurun_out/exp14/pytest_m16.log; [ $rc -ne 0 ] && exit $rc
for m in 12 16 17; do
  MTSG_TRACE_MODE=$m run "m$m" 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
done
for m in 16; do
  MTSG_TRACE_MODE=$m run "m${m}_c5" 400 python bench.py --workload c5 --width 1920 --height 1080 --spp 64 --steps 2 --warmup 1 --no-cpu || exit $?
done
