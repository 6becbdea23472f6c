#!/bin/bash
# GPU-box session: parity tests, smoke, short bench.  Each GPU step has its own
# time limit; any fault/abort/timeout (exit >= 2 from pytest, != 0 otherwise)
# ends the script.
mkdir -p gpurun_out
run() {   # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n ${TAILN:-25} "gpurun_out/$name.log"
  return $rc
}
run pytest_gpu 400 python -m pytest tests -q -m gpu; rc=$?
if [ $rc -ge 2 ]; then exit $rc; fi
TAILN=12 run parity_glass 200 python tools/parity_report.py scenes/cbox_glass.xml width=48 height=48 spp=8 || exit $?
TAILN=12 run parity_glass256 300 python tools/parity_report.py scenes/cbox_glass.xml width=48 height=48 spp=256 || exit $?
run bench_cbox 300 python bench.py --workload cbox --steps 2 --warmup 1 --no-cpu || exit $?
run bench_bunny 400 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
