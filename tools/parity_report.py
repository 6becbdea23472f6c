#!/usr/bin/env python3
"""Per-pixel parity report: GPU (libmtsg) vs CPU oracle, counter-mode RNG.
usage: python tools/parity_report.py scene.xml [name=value ...] [--glass]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "my-mitsuba_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import mtsg  # noqa: E402
from oracle import pyoracle as O  # noqa: E402


def main():
    path = sys.argv[1]
    defs = dict(a.split("=", 1) for a in sys.argv[2:] if "=" in a)
    scene = mtsg.Scene(path, defs)
    p = scene.params()
    b = scene.border
    g = mtsg.GPUScene(scene, 0)
    img_g = g.render(p, b)
    img_c, _ = O.render(scene.desc, p, b, rng=O.RNG_COUNTER)
    rgb_g, rgb_c = mtsg.develop(img_g), mtsg.develop(img_c)
    d = np.abs(rgb_g - rgb_c).max(-1)
    mean = rgb_c.mean()
    print(f"{path} {defs}: mean radiance {mean:.5f}  mean L1 {np.abs(rgb_g - rgb_c).mean():.3e}  "
          f"rel {np.abs(rgb_g - rgb_c).mean() / mean:.3e}")
    for thr in (1e-6, 1e-4, 1e-2, 1e-1):
        print(f"  pixels with max|diff| > {thr:g}: {(d > thr).mean() * 100:.3f}%")
    iy, ix = np.unravel_index(np.argmax(d), d.shape)
    print(f"  worst pixel ({ix},{iy}) block-coords: gpu {rgb_g[iy, ix]} cpu {rgb_c[iy, ix]}")
    print(f"  weight channel max rel diff: {np.nanmax(np.abs(img_g[..., 4] - img_c[..., 4]) / np.maximum(img_c[..., 4], 1e-12)):.3e}")
    g.close()


if __name__ == "__main__" and "--samples" not in sys.argv and "--replay" not in sys.argv:
    main()


def samples_diff(path, defs, maxshow=12):
    """Per-sample comparison (GPU mtsg_render_samples vs oracle_pixel_samples)."""
    scene = mtsg.Scene(path, defs)
    p = scene.params()
    g = mtsg.GPUScene(scene, 0)
    Lg = g.render_samples(p)
    shown = 0
    ndiff = 0
    for y in range(p.tile_h):
        for x in range(p.tile_w):
            Lc = O.pixel_samples(scene.desc, p, p.tile_x + x, p.tile_y + y)
            d = np.abs(Lg[y, x, :, :3] - Lc).max(-1)
            bad = np.nonzero(d > 1e-3 * (np.abs(Lc).max(-1) + 1e-3))[0]
            ndiff += len(bad)
            for s in bad:
                if shown < maxshow:
                    print(f"  sample pixel=({p.tile_x + x},{p.tile_y + y}) s={s}: gpu {Lg[y, x, s, :3]} cpu {Lc[s]}")
                    shown += 1
    print(f"  diverging samples: {ndiff} / {p.tile_w * p.tile_h * p.spp}")
    g.close()


if __name__ == "__main__" and "--samples" in sys.argv:
    args = [a for a in sys.argv[1:] if a != "--samples"]
    samples_diff(args[0], dict(a.split("=", 1) for a in args[1:] if "=" in a))


def replay(path, defs, cases):
    """Replay the oracle's closest-hit rays of diverging samples on the GPU."""
    import ctypes as C
    scene = mtsg.Scene(path, defs)
    p = scene.params()
    g = mtsg.GPUScene(scene, 0)
    L = O.lib()
    L.oracle_debug_path_rays.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]
    for (x, y, s) in cases:
        buf = np.zeros((64, 8), np.float32)
        n = L.oracle_debug_path_rays(scene.desc, C.byref(p), x, y, s, buf.ctypes.data, 64)
        rays = buf[:n]
        t0, u0, v0, p0 = O.trace_closest(scene.desc, rays)
        t1, u1, v1, p1 = g.trace_closest(rays)
        print(f"  sample ({x},{y},{s}): {n} rays")
        for i in range(n):
            flag = "" if (p0[i] == p1[i] and (t0[i] == t1[i] or abs(t0[i] - t1[i]) < 1e-6 * abs(t0[i]))) else "  <-- DIFF"
            print(f"    ray {i}: cpu prim {p0[i]:#x} t {t0[i]:.9g} | gpu prim {p1[i]:#x} t {t1[i]:.9g}{flag}")
    g.close()


if __name__ == "__main__" and "--replay" in sys.argv:
    replay(sys.argv[1], dict(a.split("=", 1) for a in sys.argv[2:] if "=" in a),
           [(14, 21, 0), (1, 20, 3), (12, 21, 6), (9, 16, 0)])
