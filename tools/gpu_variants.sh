#!/bin/bash
# C3 bench (whole frame and the emulated 8-rank share) of the default library
# and each build/var/ variant (no CPU leg)
mkdir -p gpurun_out/var
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/var/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/var/$name.log)"; return $rc; }
E=${EMU:-8}
run default 300 python bench.py --steps 3 --warmup 1 --no-cpu || exit $?
run default_e$E 300 python bench.py --steps 5 --warmup 1 --no-cpu --emulate-ranks $E || exit $?
for f in build/var/libmtsg_*.so; do
  v=$(basename $f .so); v=${v#libmtsg_}
  MTSG_LIB=$f run "$v" 300 python bench.py --steps 3 --warmup 1 --no-cpu || exit $?
  MTSG_LIB=$f run "${v}_e$E" 300 python bench.py --steps 5 --warmup 1 --no-cpu --emulate-ranks $E || exit $?
done
