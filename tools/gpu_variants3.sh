#!/bin/bash
# A/B of device-library variants on the C3 bench (no CPU / parity legs):
#   tools/gpu_variants3.sh default noguard ldstop default ...
# BENCH_ARGS (environment) adds bench.py arguments, e.g. "--instancing two-level"
O=gpurun_out/var3; mkdir -p $O
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then unset MTSG_LIB; else export MTSG_LIB=my-mitsuba_amd/var/libmtsg_$v.so; fi
  tag=$v${BENCH_ARGS:+_$(echo $BENCH_ARGS | tr -c 'a-z0-9' _)}
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --no-parity --no-count $BENCH_ARGS > $O/$tag.log 2>&1; rc=$?
  echo "$tag rc=$rc $(grep -o '"value": [0-9.]*' $O/$tag.log) $(grep -o '"trace_ms": [0-9.]*' $O/$tag.log)"
  if [ $rc -ne 0 ]; then tail -3 $O/$tag.log; exit $rc; fi
done
