#!/bin/bash
# GPU parity tests, then the C3 bench (whole frame and the emulated 8-rank share)
O=gpurun_out/quick; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }; tail -3 $O/pytest.log
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu > $O/e1.log 2>&1 || { tail $O/e1.log; exit 1; }; python tools/summarize_bench.py $O/e1.log
timeout -k 10 200 python bench.py --steps 6 --warmup 1 --no-cpu --emulate-ranks 8 > $O/e8.log 2>&1 || { tail $O/e8.log; exit 1; }; python tools/summarize_bench.py $O/e8.log
