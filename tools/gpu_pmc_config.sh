#!/bin/bash
# rocprofv3 set of one bench configuration: kernel stats, then FETCH_SIZE,
# WRITE_SIZE and TCC hit/miss in separate --pmc passes of one step each,
# summarised per kernel and keyed by the configuration (tools/pmc_kernels.py).
#   tools/gpu_pmc_config.sh r03 c3 [bench.py args...]
R=$1; TAG=$2; shift 2
O=gpurun_out/pmc_${R}_${TAG}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $TAG $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -n 5 "$O/$name.log"; exit $rc; fi; }
ARGS="--no-cpu --no-parity --no-count $*"
# --pmc-pass: each run renders only the frames it is normalised by (4 for the
# stats pass, 1 for each counter pass; share 0 of the stride deal when shares
# are emulated), so per-frame figures are per frame
step stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o stats -- python bench.py $ARGS --pmc-pass --steps 3 --warmup 1
step fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O -o fetch -- python bench.py $ARGS --pmc-pass --steps 1 --warmup 0
step write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O -o write -- python bench.py $ARGS --pmc-pass --steps 1 --warmup 0
step tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O -o tcc -- python bench.py $ARGS --pmc-pass --steps 1 --warmup 0
KEY=$(python bench.py $ARGS --print-pmc-key)
python tools/pmc_kernels.py $O "$KEY" --frames-stats 4 --frames-pass 1 > $O/pmc.json && echo "pmc summary: $O/pmc.json" || exit 1
# into this (scratch) copy's profiles/, so the bench lines of the same call
# quote the set (bench.py reads the newest committed rNN_pmc_*.json)
cp $O/pmc.json profiles/${R}_pmc_${TAG}.json
