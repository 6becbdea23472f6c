#!/bin/bash
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n ${TAILN:-12} "gpurun_out/$name.log"; return $rc; }
TAILN=8 MTSG_LIB=libmtsg_nofma.so run parity_glass_nofma 200 python tools/parity_report.py scenes/cbox_glass.xml width=48 height=48 spp=8 || exit $?
TAILN=8 MTSG_LIB=libmtsg_nofma.so run parity_cbox_nofma 200 python tools/parity_report.py scenes/cbox.xml width=64 height=48 spp=8 || exit $?
TAILN=8 run parity_cbox 200 python tools/parity_report.py scenes/cbox.xml width=64 height=48 spp=8 || exit $?
for m in 0 1 2 3; do
  for w in bunny15 cbox; do
    MTSG_TRACE_MODE=$m TAILN=1 run "mode${m}_$w" 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu || exit $?
  done
done
