O=gpurun_out/libs2; mkdir -p $O
run() { local name=$1; shift; timeout -k 10 200 "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(python tools/summarize_bench.py $O/$name.log)"; return $rc; }
for rep in 1 2; do
for lib in default my-mitsuba_amd/var_*.so; do
  v=$(basename $lib .so)
  if [ $lib = default ]; then unset MTSG_LIB; else export MTSG_LIB=$lib; fi
  run ${v}_e1_$rep python bench.py --steps 3 --warmup 1 --no-cpu || exit $?
  run ${v}_e8_$rep python bench.py --steps 6 --warmup 1 --no-cpu --emulate-ranks 8 || exit $?
done; done
