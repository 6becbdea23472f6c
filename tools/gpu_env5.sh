#!/bin/bash
mkdir -p gpurun_out/env
for lib in default nofma; do
  L=""; [ $lib != default ] && L=build/var/libmtsg_$lib.so
  MTSG_LIB=$L timeout -k 10 300 python tools/parity_report.py scenes/env_glass.xml width=64 height=36 spp=8 maxDepth=16 > gpurun_out/env/parity_$lib.log 2>&1 || exit $?
  echo $lib; head -3 gpurun_out/env/parity_$lib.log
  MTSG_LIB=$L timeout -k 10 300 python tools/parity_report.py --samples scenes/env_glass.xml width=64 height=36 spp=8 maxDepth=16 > gpurun_out/env/samples_$lib.log 2>&1 || exit $?
  tail -1 gpurun_out/env/samples_$lib.log
done
