#!/bin/bash
mkdir -p gpurun_out/exp11
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/exp11/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/exp11/$name.log)"; return $rc; }
run default 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
for v in w8 s5 s8; do
  MTSG_LIB=build/var/libmtsg_$v.so run "$v" 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
done
