#!/bin/bash
# kd-tree build parameter sweep on the GPU (MTSH_KD_* overrides of the
# gkdtree.h:734-744 defaults): whole-frame C3 and the 1/8 tile share (C4
# rehearsal) per setting.
O=gpurun_out/kdsweep
mkdir -p $O
run() {
  local tag=$1; shift
  for e in 1 8; do
    env "$@" timeout -k 10 200 python bench.py --no-cpu --no-parity --steps 3 --warmup 1 --emulate-ranks $e > $O/${tag}_e$e.log 2>&1 || { echo "$tag e$e failed"; tail -3 $O/${tag}_e$e.log; exit 1; }
    python - $O/${tag}_e$e.log $tag $e <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = j["roofline"]
print(f"{sys.argv[2]:>14s} e{sys.argv[3]}: {j['value']:9.1f} Msamples/s  {j['ms_per_step']:7.2f} ms  trace {j['kernels']['trace_ms']:7.2f} ms  "
      f"nodes {r['nodes_per_closest_ray']:.2f} tests {r['tests_per_closest_ray']:.2f}", flush=True)
PY
  done
}
if [ -n "$KD_SWEEP" ]; then eval "$KD_SWEEP"; exit 0; fi
run default X=1
run stop3 MTSH_KD_STOP_PRIMS=3
run stop4 MTSH_KD_STOP_PRIMS=4
run stop8 MTSH_KD_STOP_PRIMS=8
run trav10 MTSH_KD_TRAVERSAL=10
run trav25 MTSH_KD_TRAVERSAL=25
run trav40 MTSH_KD_TRAVERSAL=40
run empty08 MTSH_KD_EMPTY_BONUS=0.8
run empty10 MTSH_KD_EMPTY_BONUS=1.0
run noretract MTSH_KD_RETRACT=0
run trav60 MTSH_KD_TRAVERSAL=60
run trav40s3 MTSH_KD_TRAVERSAL=40 MTSH_KD_STOP_PRIMS=3
