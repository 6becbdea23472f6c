#!/bin/bash
# Tail-mode (k_finish) sweep: GPU tests with every bounce >= 1 in k_finish,
# then the whole frame and the emulated 8-rank share at several thresholds,
# and a bit-identity check of the saved images against tail mode off.
#   tools/gpu_finish.sh [thresholds...]
O=gpurun_out/fin; mkdir -p $O
TH=${*:-"0 262144 1048576 4194304"}
MTSG_FINISH=4294967295 timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest_allfinish.log 2>&1 || { tail -40 $O/pytest_allfinish.log; exit 1; }
tail -2 $O/pytest_allfinish.log
for f in $TH; do
  MTSG_FINISH=$f timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu --no-parity --emulate-ranks 8 --save $O/e8_$f.npy > $O/e8_$f.log 2>&1 || { tail $O/e8_$f.log; exit 1; }
  echo "e8 fin=$f: $(python tools/summarize_bench.py $O/e8_$f.log)"
done
for f in 0 $(echo $TH | awk '{print $NF}'); do
  MTSG_FINISH=$f timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-parity --save $O/e1_$f.npy > $O/e1_$f.log 2>&1 || { tail $O/e1_$f.log; exit 1; }
  echo "e1 fin=$f: $(python tools/summarize_bench.py $O/e1_$f.log)"
done
python - <<PY
import numpy as np, glob
for pre in ("e8", "e1"):
    fs = sorted(glob.glob("$O/%s_*.npy" % pre))
    ref = np.load("$O/%s_0.npy" % pre)
    for f in fs:
        a = np.load(f)
        print(pre, f, "bit-identical" if np.array_equal(a, ref) else "DIFFERS max %g" % np.abs(a - ref).max())
PY
