#!/bin/bash
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n ${TAILN:-12} "gpurun_out/$name.log"; return $rc; }
TAILN=6 run pytest_gpu 400 python -m pytest tests -q -m gpu; rc=$?
if [ $rc -ge 2 ]; then exit $rc; fi
for m in 0 1 3; do
  for w in bunny15 cbox; do
    MTSG_TRACE_MODE=$m TAILN=1 run "mode${m}_$w" 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu || exit $?
  done
done
