#!/usr/bin/env python3
"""Traversal iterations per ray (MTSG_FLAG_COUNT): max and log2 histogram.
usage: python tools/iter_hist.py [scene] [spp]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "my-mitsuba_amd"))
import mtsg  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "bunny15"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
scene = mtsg.Scene(os.path.join(REPO, "scenes", name + ".xml"), {"width": 1280, "height": 720, "spp": spp, "maxDepth": 8})
p = scene.params()
g = mtsg.GPUScene(scene, 0)
b = scene.border
nbytes = (p.tile_w + 2 * b) * (p.tile_h + 2 * b) * 5 * 4
film = g.alloc(nbytes)
g.set_flags(mtsg.MTSG_FLAG_COUNT)
g.render_device(p, film)
st = g.stats()
for kind in ("closest", "shadow"):
    h = list(getattr(st, "iter_hist_" + kind))
    tot = max(1, sum(h))
    print(f"{kind}: rays {tot} max iterations {getattr(st, 'iter_max_' + kind)}")
    for k, c in enumerate(h):
        if c:
            print(f"  [{1 << k:6d}, {2 << k:6d}): {c:12d}  {c / tot:.2e}")
import ctypes as C  # noqa: E402
import numpy as np  # noqa: E402
buf = np.zeros((64, 12), np.float32)
n = mtsg.device_lib().mtsg_debug_stragglers(g._h, C.c_void_p(buf.ctypes.data), 64)
print(f"stragglers captured: {n}")
for r in buf[:min(n, 64)]:
    print("  o %9.4f %9.4f %9.4f  d %8.5f %8.5f %8.5f  iters %4d %-7s nodes %4d tests %4d restarts %3d"
          % (*r[:6], r[6], "shadow" if r[7] else "closest", r[8], r[9], r[10]))
np.save(os.path.join(REPO, "gpurun_out", "stragglers.npy"), buf[:min(n, 64)])
g.free(film)
g.close()
