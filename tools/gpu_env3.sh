#!/bin/bash
mkdir -p gpurun_out/env
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "envmap_lookup" > gpurun_out/env/lookup.log 2>&1; rc=$?
tail -n 30 gpurun_out/env/lookup.log | cut -c1-300
exit $rc
