#!/bin/bash
# GPU parity tests + C3 and C5 benches (no CPU leg)
mkdir -p gpurun_out/bench
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/bench/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/bench/$name.log)"; return $rc; }
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/bench/pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/bench/pytest.log; [ $rc -ne 0 ] && exit $rc
run c3 300 python bench.py --steps 3 --warmup 1 --no-cpu || exit $?
run c5 400 python bench.py --workload c5 --width 1920 --height 1080 --spp 64 --steps 2 --warmup 1 --no-cpu || exit $?
