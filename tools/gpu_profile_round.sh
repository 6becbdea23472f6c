#!/bin/bash
# Round profile set (copied to profiles/ afterwards):
#   1. the default bench line (with the CPU baseline leg)
#   2. rocprofv3 --kernel-trace --stats of the same bench command
#   3. FETCH_SIZE and WRITE_SIZE passes (separate --pmc runs) -> HBM traffic
R=${1:-r01}
O=gpurun_out/prof_$R
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 2 "$O/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step bench 600 python bench.py
step stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o stats -- python bench.py --no-cpu
step fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O -o fetch -- python bench.py --no-cpu --steps 1 --warmup 0
step write 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O -o write -- python bench.py --no-cpu --steps 1 --warmup 0
python tools/traffic_summary.py $O > $O/traffic.json && cat $O/traffic.json
