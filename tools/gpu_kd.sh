#!/bin/bash
# device kd build tests (-s: print the C3 build times), then C3 rendered
# through the device-built tree
O=gpurun_out/kd
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kdbuild.py -x -v -s --timeout 300 --timeout-method thread > $O/kd.log 2>&1; rc=$?
grep -E "device build|PASS|FAIL|Error|error" $O/kd.log | head -30
tail -n 3 $O/kd.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu --no-parity --kd-build device > $O/bench_kd.log 2>&1; rc=$?
tail -c 1500 $O/bench_kd.log
exit $rc
