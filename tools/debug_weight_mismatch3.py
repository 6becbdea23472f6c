#!/usr/bin/env python3
"""Render single pixels around a weight mismatch on both sides and compare the
5x5 ImageBlocks, printing the pixel jitters (splat arithmetic check)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "my-mitsuba_amd"), REPO]
import mtsg  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

np.set_printoptions(precision=9, linewidth=200)
scene = mtsg.Scene(os.path.join(REPO, "scenes/bunny15.xml"), {"width": 1280, "height": 720, "spp": 2})
g = mtsg.GPUScene(scene, 0)
b = scene.border
for y in range(28, 33):
    for x in range(753, 758):
        pp = scene.params(tile_x=x, tile_y=y, tile_w=1, tile_h=1)
        bg = g.render(pp, b)[..., 4]
        bc, _ = O.render(scene.desc, pp, b, rng=O.RNG_COUNTER)
        bc = bc[..., 4]
        if not np.allclose(bg, bc, rtol=1e-6, atol=1e-7):
            print(f"pixel ({x},{y}) jitters:", [g.sampler_draws(pp, x, y, s, [2]) for s in range(2)],
                  [O.sampler_draws(scene.desc, pp, x, y, s, [2]) for s in range(2)])
            print(" gpu\n", bg, "\n oracle\n", bc)
# the same pixel inside its full 16x16 tile vs alone
g.close()
