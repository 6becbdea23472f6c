#!/bin/bash
# Session-start check: GPU tests, the default bench line, the two-level C3
# variant and the emulated 1/8 (C4, 8-rank) share.
O=gpurun_out/check
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 3 "$O/$name.log" | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
for w in ${*:-tests bench inst e8}; do
  case $w in
    tests) step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 3 ;;
    inst) step inst 300 python bench.py --steps 5 --warmup 2 --instancing two-level --no-cpu --no-parity ;;
    e8) step e8 300 python bench.py --steps 10 --warmup 3 --emulate-ranks 8 --no-cpu --no-parity ;;
  esac
done
