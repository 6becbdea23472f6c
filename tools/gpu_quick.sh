#!/bin/bash
# GPU parity tests + default benches (no CPU leg)
mkdir -p gpurun_out/quick
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/quick/pytest_gpu.log 2>&1; rc=$?; tail -n 2 gpurun_out/quick/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for w in bunny15 cbox; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --workload $w > gpurun_out/quick/bench_$w.log 2>&1 || exit $?
  echo "$w $(python tools/summarize_bench.py gpurun_out/quick/bench_$w.log)"
done
