#!/bin/bash
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n ${TAILN:-12} "gpurun_out/$name.log"; return $rc; }
TAILN=14 run samples_glass 200 python tools/parity_report.py scenes/cbox_glass.xml width=24 height=24 spp=8 --samples || exit $?
for bp in 4194304 16777216 33554432; do
  for m in 0 3; do
    MTSG_TRACE_MODE=$m TAILN=1 run "bp${bp}_m${m}_bunny" 300 python bench.py --workload bunny15 --steps 2 --warmup 1 --no-cpu --batch-paths $bp || exit $?
  done
done
MTSG_TRACE_MODE=0 TAILN=1 run "bp33554432_m0_cbox" 300 python bench.py --workload cbox --steps 2 --warmup 1 --no-cpu --batch-paths 33554432 || exit $?
MTSG_TRACE_MODE=3 TAILN=1 run "bp33554432_m3_cbox" 300 python bench.py --workload cbox --steps 2 --warmup 1 --no-cpu --batch-paths 33554432 || exit $?
