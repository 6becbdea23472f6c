#!/bin/bash
mkdir -p gpurun_out/exp12
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/exp12/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/exp12/$name.log)"; return $rc; }
for lib in default nofma; do
  L=""; [ $lib != default ] && L=build/var/libmtsg_$lib.so
  MTSG_LIB=$L run "c3_$lib" 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
  MTSG_LIB=$L run "c5_$lib" 400 python bench.py --workload c5 --width 1920 --height 1080 --spp 64 --steps 2 --warmup 1 --no-cpu || exit $?
done
