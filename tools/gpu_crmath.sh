#!/bin/bash
# A/B of the float transcendentals (default) against double-evaluated sincos
# (variant crsc, MTSG_CR_MATH=1): GPU tests, then C5 and C3 bench lines with
# their parity legs.
O=gpurun_out/crmath; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 2 "$O/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
V=my-mitsuba_amd/var/libmtsg_crsc.so
step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
MTSG_LIB=$V step tests_crsc 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
C5="--workload c5 --width 1920 --height 1080 --spp 1024 --no-cpu --no-count"
MTSG_LIB=$V step c5_crsc 300 python bench.py --steps 3 --warmup 1 $C5
step c5_fl 300 python bench.py --steps 3 --warmup 1 $C5
MTSG_LIB=$V step c3_crsc 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-count
step c3_fl 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-count
