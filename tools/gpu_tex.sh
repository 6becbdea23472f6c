#!/bin/bash
# texture GPU tests, then the default bench line
O=gpurun_out/tex
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_textures.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -n 15 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu > $O/bench.log 2>&1; rc=$?
tail -c 600 $O/bench.log
exit $rc
