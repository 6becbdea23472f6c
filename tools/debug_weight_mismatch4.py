#!/usr/bin/env python3
"""Which side changes with the render rectangle: a window around the
mismatching texels rendered as its own rectangle vs cut out of the full frame,
for the GPU and for the oracle."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "my-mitsuba_amd"), REPO]
import mtsg  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

np.set_printoptions(precision=8, linewidth=220)
scene = mtsg.Scene(os.path.join(REPO, "scenes/bunny15.xml"), {"width": 1280, "height": 720, "spp": 2})
g = mtsg.GPUScene(scene, 0)
b = scene.border
full_g = g.render(scene.params(), b)[..., 4]
full_c = O.render(scene.desc, scene.params(), b, rng=O.RNG_COUNTER)[0][..., 4]
for (x0, y0, w, h) in [(736, 0, 64, 64), (752, 16, 16, 16), (704, 0, 128, 128)]:
    pp = scene.params(tile_x=x0, tile_y=y0, tile_w=w, tile_h=h)
    rg = g.render(pp, b)[..., 4]
    rc = O.render(scene.desc, pp, b, rng=O.RNG_COUNTER)[0][..., 4]
    # interior texels only (the rectangle's border texels miss neighbours)
    sl = (slice(y0 + 2 * b, y0 + h), slice(x0 + 2 * b, x0 + w))
    fg, fc = full_g[sl], full_c[sl]
    ig, ic = rg[2 * b:h, 2 * b:w], rc[2 * b:h, 2 * b:w]
    print(f"rect {x0},{y0},{w}x{h}: gpu rect vs gpu full {np.abs(ig - fg).max():.3e}; oracle rect vs oracle full "
          f"{np.abs(ic - fc).max():.3e}; gpu rect vs oracle rect {np.abs(ig - ic).max():.3e}")
g.close()
