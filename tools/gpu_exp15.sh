#!/bin/bash
# branch-light compact traversal: parity + C3/C5 bench
mkdir -p gpurun_out/exp15
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/exp15/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/exp15/$name.log)"; return $rc; }
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/exp15/pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/exp15/pytest.log; [ $rc -ne 0 ] && exit $rc
run c3 300 python bench.py --steps 3 --warmup 1 --no-cpu || exit $?
run c5 400 python bench.py --workload c5 --width 1920 --height 1080 --spp 64 --steps 2 --warmup 1 --no-cpu || exit $?
