#!/bin/bash
# One GPU call: GPU tests, the bench line, and the rocprof set of this round
# (kernel stats, FETCH/WRITE traffic passes, TCC hit-rate pass).
#   tools/gpu_round.sh r02 [tests|bench|prof ...]
R=${1:-r02}; shift
WHAT=${*:-tests bench prof}
O=gpurun_out/prof_$R
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 3 "$O/$name.log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
for w in $WHAT; do
  case $w in
    tests) step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 3 ;;
    prof)
      step stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o stats -- python bench.py --no-cpu --no-parity
      step fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O -o fetch -- python bench.py --no-cpu --no-parity --steps 1 --warmup 0
      step write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O -o write -- python bench.py --no-cpu --no-parity --steps 1 --warmup 0
      step tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O -o tcc -- python bench.py --no-cpu --no-parity --steps 1 --warmup 0
      python tools/traffic_summary.py $O > $O/traffic.json && cat $O/traffic.json
      python tools/tcc_summary.py $O > $O/tcc.json && cat $O/tcc.json ;;
  esac
done
