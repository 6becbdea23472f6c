#!/bin/bash
# two-level instancing: GPU tests, then the two-level C3 bench line
O=gpurun_out/inst
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_instancing.py tests/test_gpu_textures.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -n 3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 170 python bench.py --steps 5 --warmup 2 --no-cpu --no-parity --instancing two-level > $O/bench.log 2>&1; rc=$?
python3 - $O/bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); r = d["roofline"]
print(d["value"], d["ms_per_step"], d["kernels"]["trace_ms"], r["nodes_per_closest_ray"], r["tests_per_closest_ray"], r["avg_launch_ms"])
PY
exit $rc
