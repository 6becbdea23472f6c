#!/usr/bin/env python3
"""Coplanar-tie probe: the rays of tests/test_gpu_parity.py::test_coplanar_tie_policy
whose closest primitive differs between the GPU and the oracle, with both
answers (primitive, t bits) saved to gpurun_out/tie_probe.npz."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "my-mitsuba_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import mtsg  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

scene = mtsg.Scene(os.path.join(REPO, "scenes", "cbox_glass.xml"), {"width": 48, "height": 48, "spp": 8, "glassY": -0.7})
b = scene.prim_bounds()
flat = np.flatnonzero((b[:, 1] == -1.0) & (b[:, 4] == -1.0))
rng = np.random.default_rng(17)
rays = []
for p in flat[:-1]:
    n = 4000
    x = rng.uniform(b[p, 0], b[p, 3], n)
    z = rng.uniform(b[p, 2], b[p, 5], n)
    for y0, dy in ((-1.0 - 0.25, 1.0), (-1.0 + 0.05, -1.0)):
        r = np.zeros((n, 8), np.float32)
        r[:, 0], r[:, 1], r[:, 2] = x, y0, z
        d = np.stack([rng.normal(0, 0.05, n), np.full(n, dy), rng.normal(0, 0.05, n)], 1)
        r[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
        r[:, 6], r[:, 7] = 1e-4, np.inf
        rays.append(r)
rays = np.concatenate(rays)
t0, u0, v0, p0 = O.trace_closest(scene.desc, rays)
g = mtsg.GPUScene(scene, 0)
t1, u1, v1, p1 = g.trace_closest(rays)
g.close()
bad = p0 != p1
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "tie_probe.npz"), rays=rays[bad], t0=t0[bad], p0=p0[bad], t1=t1[bad], p1=p1[bad])
print("differing", int(bad.sum()), "of", len(rays), "t equal among them", int((t0[bad] == t1[bad]).sum()))
for i in np.flatnonzero(bad)[:8]:
    print(rays[i, :6], "oracle", hex(p0[i]), t0[i].view(np.uint32), "gpu", hex(p1[i]), t1[i].view(np.uint32))
