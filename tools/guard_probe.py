#!/usr/bin/env python3
"""Restart-guard probe: closest-hit disagreement with the oracle for the
corner / degenerate rays of tests/test_gpu_edge_rays.py under stack caps and
guard thresholds (environment read at mtsg_scene_create)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "my-mitsuba_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402

import mtsg  # noqa: E402
from oracle import pyoracle as O  # noqa: E402
from test_gpu_edge_rays import bounds, corner_rays, degenerate_rays, planes  # noqa: E402

SC = os.path.join(os.path.dirname(__file__), "..", "scenes")
for name in sys.argv[1:] or ["cbox", "bunny15"]:
    inst = "two-level" if name.endswith("two-level") else "flatten"
    s = mtsg.Scene(os.path.join(SC, "cbox.xml" if name == "cbox" else "bunny15.xml"), {"width": 32, "height": 24, "spp": 1},
                   instancing=inst)
    rays = np.concatenate([corner_rays(s, 30000, 51), degenerate_rays(*bounds(s), 20000, 52, planes(s))])
    t0, _, _, p0 = O.trace_closest(s.desc, rays)
    for cap, guard in (("6", "8"), ("1", "8"), ("1", "64"), ("1", "1000"), ("2", "8"), ("1", "0")):
        os.environ["MTSG_STACK_CAP"], os.environ["MTSG_RESTART_GUARD"] = cap, guard
        g = mtsg.GPUScene(s, 0)
        try:
            t1, _, _, p1 = g.trace_closest(rays)
            h0, h1 = p0 != 0xFFFFFFFF, p1 != 0xFFFFFFFF
            both = h0 & h1
            dp = both & (p0 != p1) & (np.abs(t0 - t1) > 1e-4 * np.abs(t0))
            print(f"{name} cap {cap} guard {guard}: hit/miss differ {int((h0 != h1).sum())} "
                  f"(gpu-miss {int((h0 & ~h1).sum())}, gpu-extra {int((~h0 & h1).sum())}), prim differ {int(dp.sum())} of {len(rays)}",
                  flush=True)
        except RuntimeError as e:
            print(f"{name} cap {cap} guard {guard}: {e}", flush=True)
        g.close()
