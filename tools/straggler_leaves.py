#!/usr/bin/env python3
"""Why are the straggler rays long?  Re-traverses the rays captured by
tools/iter_hist.py (gpurun_out/stragglers.npy) on the host kd-tree with a
plain front-to-back traversal and prints, per ray, the leaves visited, the
primitive references tested and how many of them repeat (a primitive that
straddles many leaves -- e.g. the ground rectangle -- is re-tested in each).
usage: python tools/straggler_leaves.py [scene] [stragglers.npy]"""
import collections
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "my-mitsuba_amd"))
import mtsg  # noqa: E402
sys.path.insert(0, os.path.join(REPO, "oracle"))
import pyoracle  # noqa: E402

P = C.c_void_p
U = C.c_uint32


class Desc(C.Structure):
    _fields_ = [("abi", U), ("nv", U), ("pos", P), ("nrm", P), ("ntri", U), ("tri_idx", P), ("dpdu", P),
                ("nrects", U), ("rects", P), ("nshapes", U), ("shapes", P), ("nbsdfs", U), ("bsdfs", P),
                ("nem", U), ("em", P), ("emcdf", P), ("nemtri", U), ("emtricdf", P),
                ("n_nodes", U), ("nodes", P), ("n_indices", U), ("indices", P), ("n_prims", U), ("triaccel", P),
                ("amin", C.c_float * 3), ("amax", C.c_float * 3), ("max_depth", U)]


def arr(ptr, n, dt):
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(dt)), shape=(n,)).copy()


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "bunny15"
    path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out", "stragglers.npy")
    scene = mtsg.Scene(os.path.join(REPO, "scenes", name + ".xml"))
    d = C.cast(scene.desc, C.POINTER(Desc)).contents
    nodes = arr(d.nodes, 2 * d.n_nodes, C.c_uint32).reshape(-1, 2)
    idx = arr(d.indices, d.n_indices, C.c_uint32)
    ta = arr(d.triaccel, 12 * d.n_prims, C.c_uint32).reshape(-1, 12)
    amin, amax = np.array(d.amin[:]), np.array(d.amax[:])
    print(f"nodes {d.n_nodes} refs {d.n_indices} prims {d.n_prims} rects {d.nrects} max depth {d.max_depth}")
    leaf = nodes[:, 0] >> 31 == 1
    sizes = (nodes[leaf, 1] - (nodes[leaf, 0] & 0x7FFFFFFF)).astype(np.int64)
    print(f"leaves {leaf.sum()} mean size {sizes.mean():.2f} max {sizes.max()} "
          f"empty {np.mean(sizes == 0):.2f}")
    rect_ids = np.nonzero(ta[:, 0] == 0xFFFFFFFF)[0]
    for r in rect_ids:
        print(f"rect prim {r}: referenced by {(idx == r).sum()} leaves")
    rays = np.load(path)
    q = np.zeros((len(rays), 8), np.float32)
    q[:, 0:6] = rays[:, 0:6]
    q[:, 7] = np.inf
    thit, _, _, phit = pyoracle.trace_closest(scene.desc, q)
    for ray, th, ph in zip(rays[:12], thit, phit):
        o, dd = ray[0:3].astype(np.float64), ray[3:6].astype(np.float64)
        inv = 1.0 / np.where(dd == 0, 1e-30, dd)
        t0s, t1s = (amin - o) * inv, (amax - o) * inv
        tmin, tmax = max(np.minimum(t0s, t1s).max(), 0.0), np.maximum(t0s, t1s).min()
        stack = [(0, tmin, tmax)]
        leaves, refs, rep = 0, 0, collections.Counter()
        deep = 0
        while stack:
            n, a, b = stack.pop()
            if a > th:
                break
            depth = 0
            while not (nodes[n, 0] >> 31):
                ax = nodes[n, 0] & 3
                split = np.frombuffer(np.uint32(nodes[n, 1]).tobytes(), np.float32)[0]
                left = n + (nodes[n, 0] >> 2)
                ts = (split - o[ax]) * inv[ax]
                near, far = (left, left + 1) if o[ax] < split or (o[ax] == split and dd[ax] <= 0) else (left + 1, left)
                if ts > b or ts <= 0:
                    n = near
                elif ts < a:
                    n = far
                else:
                    stack.append((far, ts, b))
                    n, b = near, ts
                depth += 1
            deep = max(deep, depth)
            s, e = nodes[n, 0] & 0x7FFFFFFF, nodes[n, 1]
            leaves += 1
            refs += int(e - s)
            rep.update(idx[s:e].tolist())
        dup = sum(c - 1 for c in rep.values() if c > 1)
        top = rep.most_common(3)
        print(f"d {dd.round(4)} gpu iters {int(ray[6])} nodes {int(ray[8])} tests {int(ray[9])} | "
              f"to hit t={th:.3f} prim {ph}: leaves {leaves} refs {refs} unique {len(rep)} repeats {dup} "
              f"top {top}")


if __name__ == "__main__":
    main()
