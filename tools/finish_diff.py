#!/usr/bin/env python3
"""Per-sample radiance with the tail kernel (k_finish) from bounce 1 on vs
the per-bounce kernels: count and show the samples that differ.
usage: python tools/finish_diff.py [scene] [w] [h] [spp]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "my-mitsuba_amd"))
import mtsg  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "bunny15"
w, h, spp = (int(v) for v in (sys.argv[2:5] if len(sys.argv) > 4 else (160, 90, 4)))
scene = mtsg.Scene(os.path.join(REPO, "scenes", name + ".xml"), {"width": w, "height": h, "spp": spp, "maxDepth": 8})
out = {}
for f in ("0", "4294967295"):
    os.environ["MTSG_FINISH"] = f
    g = mtsg.GPUScene(scene, 0)
    out[f] = g.render_samples(scene.params())
    g.close()
a, b = out["0"], out["4294967295"]
d = np.abs(a - b).max(axis=-1)
bad = np.argwhere(d > 0)
print(f"{name} {w}x{h}x{spp}: {len(bad)} of {d.size} samples differ, max |diff| {d.max():.3g}")
for idx in bad[:12]:
    print("  ", tuple(int(v) for v in idx), a[tuple(idx)], b[tuple(idx)])
