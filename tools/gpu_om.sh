#!/bin/bash
# OM + texture GPU tests, then the whole -m gpu suite
O=gpurun_out/om
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_om.py -x -v --timeout 300 --timeout-method thread > $O/om.log 2>&1; rc=$?
tail -n 14 $O/om.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/all.log 2>&1; rc=$?
tail -n 4 $O/all.log
exit $rc
