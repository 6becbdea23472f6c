#!/bin/bash
# C3 bench (whole frame and the emulated 8-rank share) for the default library
# and each my-mitsuba_amd/var_*.so (MTSG_LIB), with each one's wave drain profile
O=gpurun_out/libs; mkdir -p $O
run() { local name=$1; shift; timeout -k 10 200 "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py $O/$name.log)"; return $rc; }
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }; tail -1 $O/pytest.log
for lib in default my-mitsuba_amd/var_*.so; do
  v=$(basename $lib .so)
  if [ $lib = default ]; then unset MTSG_LIB; else export MTSG_LIB=$lib; fi
  timeout -k 10 100 python tools/wavetime.py bunny15 256 8 > $O/${v}_wt8.log 2>&1 || exit $?
  grep -A1 "launch  0:" $O/${v}_wt8.log | cut -c1-200
  run ${v}_e1 python bench.py --steps 3 --warmup 1 --no-cpu || exit $?
  run ${v}_e8 python bench.py --steps 6 --warmup 1 --no-cpu --emulate-ranks 8 || exit $?
done
