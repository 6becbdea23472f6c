#!/usr/bin/env python3
"""Find samples rejected on one side only (NaN / negative radiance: ImageBlock::put
drops them, imageblock.h:147-151) in a GPU-vs-oracle render: locate pixels whose
filter-weight sums differ, then compare per-sample radiance of the tile around
them (mtsg_render_samples vs oracle_pixel_samples) and trace the odd sample."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "my-mitsuba_amd"), REPO]
import mtsg  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

scene_file = sys.argv[1] if len(sys.argv) > 1 else "scenes/bunny15.xml"
w, h, spp = (int(v) for v in (sys.argv[2:5] if len(sys.argv) > 4 else (1280, 720, 2)))
scene = mtsg.Scene(os.path.join(REPO, scene_file), {"width": w, "height": h, "spp": spp})
g = mtsg.GPUScene(scene, 0)
p = scene.params()
b = scene.border
img_g = g.render(p, b)
img_c, _ = O.render(scene.desc, p, b, rng=O.RNG_COUNTER)
dw = np.abs(img_g[..., 4] - img_c[..., 4])
bad = np.argwhere(dw > 1e-5 + 1e-5 * np.abs(img_c[..., 4]))
print("weight mismatches:", len(bad), "max", dw.max())
seen = set()
for (yy, xx) in bad[:40]:
    y0, x0 = yy - b, xx - b
    for y in range(max(0, y0 - 2), min(h, y0 + 3)):
        for x in range(max(0, x0 - 2), min(w, x0 + 3)):
            if (x, y) in seen:
                continue
            seen.add((x, y))
            pp = scene.params(tile_x=x, tile_y=y, tile_w=1, tile_h=1)
            Lg = g.render_samples(pp)[0, 0, :, :3]
            Lc = O.pixel_samples(scene.desc, pp, x, y)
            for s in range(spp):
                okg = np.all(np.isfinite(Lg[s])) and np.all(Lg[s] >= 0)
                okc = np.all(np.isfinite(Lc[s])) and np.all(Lc[s] >= 0)
                if okg != okc or (okg and np.abs(Lg[s] - Lc[s]).max() > 1e-3 * (1 + np.abs(Lc[s]).max())):
                    print(f"pixel ({x},{y}) sample {s}: gpu {Lg[s]} oracle {Lc[s]}", flush=True)
                    L = O.lib()
                    L.oracle_debug_pixel_sample.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
                    L.oracle_debug_pixel_sample(scene.desc, C.byref(pp), x, y, s)
g.close()
