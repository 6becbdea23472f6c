#!/usr/bin/env python3
"""One line per bench step of a tools/gpu_r04.sh call: value and kernel times
(gpurun_out/r4/*.log, in the order of the steps' start)."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r4"
rows = []
for f in glob.glob(os.path.join(d, "*.log")):
    lines = [l for l in open(f, errors="replace") if l.startswith("{")]
    if not lines:
        continue
    try:
        j = json.loads(lines[-1])
    except ValueError:
        continue
    k = j.get("kernels", {})
    rows.append((os.path.getmtime(f), os.path.basename(f)[:-4], j.get("value"), k.get("trace_ms"), k.get("shade_ms"),
                 k.get("finish_ms"), k.get("frame_ms"), j.get("share_speedup_min")))
for _, n, v, t, s, fi, fr, sp in sorted(rows):
    f = lambda x: f"{x:8.2f}" if isinstance(x, (int, float)) else f"{'-':>8}"  # noqa: E731
    print(f"{n:24s} {f(v)} trace {f(t)} shade {f(s)} finish {f(fi)} frame {f(fr)}" + (f" min-share {sp:.3f}" if sp else ""))
