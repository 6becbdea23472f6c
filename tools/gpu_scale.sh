#!/bin/bash
# GPU tests + C3 bench at 1 GPU and the emulated 2/4/8-rank shares (one GPU, rank 0's tiles)
mkdir -p gpurun_out/scale
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/scale/pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/scale/pytest.log; [ $rc -ne 0 ] && exit $rc
for n in 1 2 4 8; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --emulate-ranks $n > gpurun_out/scale/c3_e$n.log 2>&1 || exit $?
  echo "e$n $(python tools/summarize_bench.py gpurun_out/scale/c3_e$n.log)"
done
