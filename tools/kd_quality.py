#!/usr/bin/env python3
"""Tree-quality sweep on the CPU: nodes / primitive tests per closest ray of
the oracle (counting mode) on bunny15 for kd build-parameter overrides.
usage: MTSH_KD_...=... python tools/kd_quality.py"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "my-mitsuba_amd"))
sys.path.insert(0, REPO)
import mtsg  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

t0 = time.time()
sc = mtsg.Scene(os.path.join(REPO, "scenes", "bunny15.xml"), {"width": 320, "height": 180, "spp": 4, "maxDepth": 8})
tb = time.time() - t0
p = sc.params()
_, st = O.render(sc.desc, p, sc.border, rng=O.RNG_COUNTER, count=True)
i = sc.info
print(f"build {i.kd_build_seconds:.2f}s nodes={i.kd_nodes} indices={i.kd_indices} depth={i.kd_max_depth} "
      f"| per closest ray: nodes {st.nodes_visited / st.rays_closest:.2f} tests {st.tri_tests / st.rays_closest:.2f} "
      f"| per ray (closest+shadow): {(st.nodes_visited + st.tri_tests) / (st.rays_closest + st.rays_shadow):.2f} iters "
      f"| render {st.seconds:.2f}s")
