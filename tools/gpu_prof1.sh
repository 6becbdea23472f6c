#!/bin/bash
mkdir -p gpurun_out/prof
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n ${TAILN:-12} "gpurun_out/$name.log"; return $rc; }
TAILN=14 run samples_glass 200 python tools/parity_report.py scenes/cbox_glass.xml width=24 height=24 spp=8 --samples || exit $?
TAILN=3 run counters_list 60 rocprofv3 -L || true
export TMPDIR=/tmp
TAILN=40 run prof_bunny 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bunny --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu || exit $?
ls -la gpurun_out/prof gpurun_out/prof/* | head -30
