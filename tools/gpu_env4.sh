#!/bin/bash
mkdir -p gpurun_out/env
for md in 16 4 3; do
timeout -k 10 300 python tools/parity_report.py --samples scenes/env_glass.xml width=64 height=36 spp=8 maxDepth=$md > gpurun_out/env/samples_md$md.log 2>&1 || exit $?
echo "maxDepth $md"; tail -6 gpurun_out/env/samples_md$md.log
done
