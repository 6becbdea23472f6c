#!/bin/bash
# A/B of device-library variants on the C3 bench (no CPU / parity legs):
#   tools/gpu_variants3.sh default noguard ldstop default ...
O=gpurun_out/var3; mkdir -p $O
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then unset MTSG_LIB; else export MTSG_LIB=my-mitsuba_amd/var/libmtsg_$v.so; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --no-parity --no-count > $O/$v.log 2>&1; rc=$?
  echo "$v rc=$rc $(grep -o '"value": [0-9.]*' $O/$v.log) $(grep -o '"trace_ms": [0-9.]*' $O/$v.log)"
  if [ $rc -ne 0 ]; then tail -3 $O/$v.log; exit $rc; fi
done
