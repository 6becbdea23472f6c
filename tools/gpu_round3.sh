#!/bin/bash
# Round-3 GPU call: tests, the default bench line, the two-level C3 line, the
# emulated 8-rank shares, then keyed PMC sets (tools/gpu_pmc_config.sh).
#   tools/gpu_round3.sh [tests] [bench] [inst] [e8] [pmc-c3] [pmc-inst] [pmc-c5] [pmc-e8]
O=gpurun_out/r3
mkdir -p $O
export TMPDIR=/tmp
# a step that fails stops the call, except test failures (pytest rc 1): the
# GPU is fine then and the other steps still run
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 3 "$O/$name.log" | cut -c1-800; if [ $rc -ne 0 ] && ! { [ "$name" = tests ] && [ $rc -eq 1 ]; }; then exit $rc; fi; }
for w in ${*:-tests bench inst e8}; do
  case $w in
    tests) step tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    kd) step kd 300 python bench.py --steps 5 --warmup 2 --kd-build device --no-cpu --no-parity ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 3 ;;
    inst) step inst 300 python bench.py --steps 5 --warmup 2 --instancing two-level --no-cpu --no-parity ;;
    e8) step e8 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 --no-cpu --no-parity ;;
    c5) step c5 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 ;;
    c2) step c2 600 python bench.py --steps 5 --warmup 2 --workload cbox ;;
    pmc-c3) bash tools/gpu_pmc_config.sh r03 c3 || exit $? ;;
    pmc-inst) bash tools/gpu_pmc_config.sh r03 c3_two_level --instancing two-level || exit $? ;;
    pmc-c5) bash tools/gpu_pmc_config.sh r03 c5 --workload c5 --width 1920 --height 1080 --spp 1024 || exit $? ;;
    pmc-e8) bash tools/gpu_pmc_config.sh r03 c4_share8 --emulate-ranks 8 || exit $? ;;
  esac
done
