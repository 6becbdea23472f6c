#!/bin/bash
# batch balancing, NT default, leaf prefetch; batch size sweep
mkdir -p gpurun_out/exp5
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/exp5/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py gpurun_out/exp5/$name.log)"; return $rc; }
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/exp5/pytest_gpu.log 2>&1; rc=$?; tail -n 2 gpurun_out/exp5/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for lib in default nont pf pfw5; do
  L=""; [ $lib != default ] && L=build/var/libmtsg_$lib.so
  MTSG_LIB=$L run "${lib}" 300 python bench.py --steps 2 --warmup 1 --no-cpu || exit $?
done
for bp in 67108864 134217728; do
  run "bp$bp" 300 python bench.py --steps 2 --warmup 1 --no-cpu --batch-paths $bp || exit $?
  MTSG_LIB=build/var/libmtsg_pf.so run "pf_bp$bp" 300 python bench.py --steps 2 --warmup 1 --no-cpu --batch-paths $bp || exit $?
done
run cbox_bp67108864 300 python bench.py --steps 2 --warmup 1 --no-cpu --workload cbox --batch-paths 67108864 || exit $?
