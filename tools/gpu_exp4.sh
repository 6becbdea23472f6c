#!/bin/bash
# A/B matrix: streaming state access, occupancy (short-stack size), leaf layout, batch size
mkdir -p gpurun_out/exp4
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/exp4/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/exp4/$name.log)"; return $rc; }
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/exp4/pytest_gpu.log 2>&1; rc=$?; tail -n 3 gpurun_out/exp4/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
MTSG_TRACE_MODE=4 timeout -k 10 300 python -m pytest tests -q -m gpu -x -k "render or dielectric" > gpurun_out/exp4/pytest_mode4.log 2>&1 || exit $?
tail -n 1 gpurun_out/exp4/pytest_mode4.log
MTSG_LIB=build/var/libmtsg_nt.so timeout -k 10 300 python -m pytest tests -q -m gpu -x -k "render or dielectric" > gpurun_out/exp4/pytest_nt.log 2>&1 || exit $?
tail -n 1 gpurun_out/exp4/pytest_nt.log
for lib in default nt s6w8 s4w8 nts6w8; do
  L=""; [ $lib != default ] && L=build/var/libmtsg_$lib.so
  for m in 3 4; do
    MTSG_LIB=$L MTSG_TRACE_MODE=$m run "${lib}_m$m" 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
  done
done
for bp in 16777216 67108864; do
  run "bp$bp" 300 python bench.py --steps 2 --warmup 1 --no-cpu --batch-paths $bp || exit $?
done
