#!/usr/bin/env python3
"""One-line summary of a bench.py JSON log (value and per-kernel ms)."""
import json
import sys

for path in sys.argv[1:]:
    line = ""
    for l in open(path):
        if l.startswith("{"):
            line = l
    if not line:
        print("no-json")
        continue
    j = json.loads(line)
    k = j.get("kernels", {})
    r = j.get("roofline") or {}
    tr = k.get("trace_ms", k.get("trace_closest_ms", 0) + k.get("trace_shadow_ms", 0))
    print(f"{j['value']:.1f} Ms/s  trace {tr:.1f} "
          f"shade {k.get('shade_ms', 0):.1f} splat {k.get('splat_ms', 0):.1f} cam {k.get('camera_ms', 0):.1f} "
          f"fin {k.get('finish_ms', 0):.2f}/{k.get('finish_paths', 0)} "
          f"frame {k.get('frame_ms', 0):.1f}  GB/s {r.get('achieved', 0)}")
