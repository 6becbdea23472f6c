#!/bin/bash
# GPU tests, then C3 at 1 GPU and the emulated 8-rank share with 1 and 2 lanes
mkdir -p gpurun_out/lanes
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/lanes/pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/lanes/pytest.log; [ $rc -ne 0 ] && exit $rc
for e in ${EMUS:-1 8}; do
  for l in ${LANES:-1 2}; do
    MTSG_LANES=$l timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --emulate-ranks $e ${EXTRA} > gpurun_out/lanes/c3_e${e}_l$l.log 2>&1 || exit $?
    echo "e$e lanes$l $(python tools/summarize_bench.py gpurun_out/lanes/c3_e${e}_l$l.log)"
  done
done
