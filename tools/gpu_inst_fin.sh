#!/bin/bash
# two-level scenes through the tail kernel: instancing / finish / render-entry GPU
# tests, then the two-level and flattened C3 frames
O=gpurun_out/instfin
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 2 "$O/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 400 python -u -m pytest tests/test_gpu_instancing.py tests/test_gpu_finish.py tests/test_gpu_textures.py tests/test_gpu_edge_rays.py -x -v --timeout 120 --timeout-method thread
step two 170 python bench.py --steps 5 --warmup 2 --no-cpu --no-parity --instancing two-level
python tools/summarize_bench.py $O/two.log
step flat 170 python bench.py --steps 5 --warmup 2 --no-cpu --no-parity
python tools/summarize_bench.py $O/flat.log
