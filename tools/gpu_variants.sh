#!/bin/bash
# C3 bench of the default library and each build/var/ variant (no CPU leg)
mkdir -p gpurun_out/var
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/var/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/var/$name.log)"; return $rc; }
run default 300 python bench.py --steps 3 --warmup 1 --no-cpu || exit $?
for f in build/var/libmtsg_*.so; do
  v=$(basename $f .so); v=${v#libmtsg_}
  MTSG_LIB=$f run "$v" 300 python bench.py --steps 3 --warmup 1 --no-cpu || exit $?
done
