#!/usr/bin/env python3
"""Render one frame of a benchmark scene on cuda:0 (for rocprofv3 runs).
usage: python tools/prof_frame.py [bunny15|cbox] [spp] [frames] [tile_stride] [flatten|two-level]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "my-mitsuba_amd"))
import mtsg  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "bunny15"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 256
frames = int(sys.argv[3]) if len(sys.argv) > 3 else 1
inst = sys.argv[5] if len(sys.argv) > 5 else "flatten"
scene = mtsg.Scene(os.path.join(REPO, "scenes", name + ".xml"), {"width": 1280, "height": 720, "spp": spp, "maxDepth": 8},
                   instancing=inst)
p = scene.params()
stride = int(sys.argv[4]) if len(sys.argv) > 4 else 1
p.tile_stride = stride
p.tile_offset = 0
g = mtsg.GPUScene(scene, 0)
b = scene.border
nbytes = (p.tile_w + 2 * b) * (p.tile_h + 2 * b) * 5 * 4
film = g.alloc(nbytes)
for _ in range(frames):
    t0 = time.perf_counter()
    g.render_device(p, film)
    dt = time.perf_counter() - t0
    print(f"{name} {spp}spp frame {dt * 1e3:.1f} ms, {p.tile_w * p.tile_h * spp / stride / dt / 1e6:.1f} Msamples/s", flush=True)
g.free(film)
g.close()
