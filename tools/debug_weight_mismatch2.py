#!/usr/bin/env python3
"""Print the texels whose filter-weight sums differ between the GPU and the
oracle, with each side's value and the splat of the samples that reach them
recomputed from the samplers' pixel jitters (imageblock.h:124-204)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "my-mitsuba_amd"), REPO]
import mtsg  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

scene = mtsg.Scene(os.path.join(REPO, "scenes/bunny15.xml"), {"width": 1280, "height": 720, "spp": 2})
g = mtsg.GPUScene(scene, 0)
p = scene.params()
b = scene.border
img_g = g.render(p, b)
img_c, _ = O.render(scene.desc, p, b, rng=O.RNG_COUNTER)
img_g2 = g.render(p, b)
print("GPU run-to-run weight max diff:", np.abs(img_g2[..., 4] - img_g[..., 4]).max(),
      "rgb:", np.abs(img_g2[..., :3] - img_g[..., :3]).max())
dw = np.abs(img_g[..., 4] - img_c[..., 4])
bad = np.argwhere(dw > 1e-5 + 1e-5 * np.abs(img_c[..., 4]))
for (yy, xx) in bad:
    print(f"texel block ({xx},{yy}) pixel ({xx-b},{yy-b}): gpu w {img_g[yy,xx,4]:.7f} oracle w {img_c[yy,xx,4]:.7f} "
          f"gpu rgb {img_g[yy,xx,:3]} oracle rgb {img_c[yy,xx,:3]}")
    for y in range(yy - b - 2, yy - b + 3):
        for x in range(xx - b - 2, xx - b + 3):
            if not (0 <= x < 1280 and 0 <= y < 720):
                continue
            pp = scene.params(tile_x=x, tile_y=y, tile_w=1, tile_h=1)
            Lg = g.render_samples(pp)[0, 0]
            for s in range(2):
                jg = g.sampler_draws(pp, x, y, s, [2])
                jc = O.sampler_draws(scene.desc, pp, x, y, s, [2])
                if not np.array_equal(jg, jc) or not np.all(np.isfinite(Lg[s])):
                    print("   jitter/L differ", x, y, s, jg, jc, Lg[s])
g.close()
