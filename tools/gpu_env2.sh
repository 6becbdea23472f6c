#!/bin/bash
mkdir -p gpurun_out/env
timeout -k 10 300 python tools/parity_report.py scenes/env_glass.xml width=64 height=36 spp=8 maxDepth=16 > gpurun_out/env/parity.log 2>&1 || exit $?
cat gpurun_out/env/parity.log
timeout -k 10 300 python tools/parity_report.py scenes/env_glass.xml width=64 height=36 spp=8 maxDepth=1 > gpurun_out/env/parity_d1.log 2>&1 || exit $?
cat gpurun_out/env/parity_d1.log
timeout -k 10 300 python tools/parity_report.py scenes/env_glass.xml width=64 height=36 spp=8 maxDepth=2 > gpurun_out/env/parity_d2.log 2>&1 || exit $?
cat gpurun_out/env/parity_d2.log
timeout -k 10 300 python tools/parity_report.py --samples scenes/env_glass.xml width=24 height=16 spp=4 maxDepth=16 > gpurun_out/env/samples.log 2>&1 || exit $?
tail -15 gpurun_out/env/samples.log
