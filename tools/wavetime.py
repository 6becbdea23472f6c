#!/usr/bin/env python3
"""Exit-time profile of the traversal waves of one frame (MTSG_FLAG_WAVETIME).
usage: python tools/wavetime.py [scene] [spp] [tile_stride]"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "my-mitsuba_amd"))
import mtsg  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "bunny15"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 256
stride = int(sys.argv[3]) if len(sys.argv) > 3 else 1
scene = mtsg.Scene(os.path.join(REPO, "scenes", name + ".xml"), {"width": 1280, "height": 720, "spp": spp, "maxDepth": 8})
p = scene.params()
p.tile_stride = stride
p.tile_offset = 0
g = mtsg.GPUScene(scene, 0)
b = scene.border
nbytes = (p.tile_w + 2 * b) * (p.tile_h + 2 * b) * 5 * 4
film = g.alloc(nbytes)
g.render_device(p, film)   # warm-up
g.set_flags(mtsg.MTSG_FLAG_WAVETIME)
g.render_device(p, film)
waves = C.c_uint32(0)
buf = np.zeros(64 * 131072 * 4, np.uint64)
n = mtsg.device_lib().mtsg_debug_wavetimes(g._h, C.c_void_p(buf.ctypes.data), 64, C.byref(waves))
W = waves.value
raw = buf[:n * W * 4].reshape(n, W, 4).astype(np.float64)
wt = raw[:, :, :3] * 10.0 / 1e3   # 100-MHz ticks -> microseconds
its = raw[:, :, 3]
np.save(os.path.join(REPO, "gpurun_out", f"wavetime_{name}_{spp}_{stride}.npy"), wt)
print(f"{name} {spp}spp stride {stride}: {n} launches x {W} waves (times in us from the launch's first wave start)")
for k in range(n):
    st, en = wt[k, :, 0], wt[k, :, 1]
    t0 = st.min()
    e = np.sort(en - t0)
    span = e[-1]
    busy = (en - st).sum() / (span * W)
    q = lambda f: e[min(W - 1, int(f * W))]  # noqa: E731
    print(f"  launch {k:2d}: span {span:8.1f}  exits 10% {q(.1):8.1f} 50% {q(.5):8.1f} 90% {q(.9):8.1f} "
          f"99% {q(.99):8.1f} 99.9% {q(.999):8.1f}  last-start {st.max() - t0:7.1f}  busy {busy:.3f}")
    # the drain: work list empty -> exit, per wave; us per loop iteration of the slowest waves
    ex = wt[k, :, 2]
    ok = ex > 0
    if ok.any():
        dr = en[ok] - ex[ok]
        it = its[k][ok]
        order = np.argsort(dr)[::-1][:16]
        first = (ex[ok] - t0).min()
        print(f"            drain: first empty {first:8.1f}  drain 50% {np.median(dr):7.1f} max {dr.max():7.1f} us; "
              f"slowest 16 waves: iters {it[order].astype(int).tolist()}  us/iter {np.round(dr[order] / np.maximum(it[order], 1), 2).tolist()}")
g.free(film)
g.close()
