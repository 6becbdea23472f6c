#!/bin/bash
mkdir -p gpurun_out/env
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/env/pytest_gpu.log 2>&1; rc=$?; tail -n 15 gpurun_out/env/pytest_gpu.log | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/parity_report.py scenes/env_glass.xml width=96 height=54 spp=16 maxDepth=16 > gpurun_out/env/parity.log 2>&1 || exit $?
tail -5 gpurun_out/env/parity.log
timeout -k 10 400 python bench.py --workload c5 --width 1920 --height 1080 --spp 64 --steps 2 --warmup 1 --no-cpu > gpurun_out/env/bench_c5.log 2>&1 || exit $?
python tools/summarize_bench.py gpurun_out/env/bench_c5.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/env/bench_c3.log 2>&1 || exit $?
python tools/summarize_bench.py gpurun_out/env/bench_c3.log
