"""Host side of the device kd-tree build: the primitive boxes handed to
mtsg_kd_build and the replacement of a scene's tree (mtsh_scene_prim_bounds,
mtsh_scene_set_kdtree).  A one-leaf tree over every live primitive is a
valid kd-tree: the oracle's Havran traversal over it must equal brute force."""
import os

import numpy as np
import pytest

import mtsg
from oracle import pyoracle as O
from conftest import SCENES


def test_prim_bounds_and_single_leaf_tree():
    s = mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {"width": 16, "height": 16, "spp": 1})
    b = s.prim_bounds()
    assert b.shape == (s.info.n_triangles + s.info.n_rects, 6)
    live = (b[:, :3] <= b[:, 3:]).all(1)
    assert live.all()
    lo, hi = b[:, :3].min(0), b[:, 3:].max(0)
    idx = np.nonzero(live)[0].astype(np.uint32)
    tree = dict(nodes=np.array([[0x80000000, idx.size]], np.uint32), indices=idx, aabb_min=lo - 1e-3, aabb_max=hi + 1e-3,
                max_depth=0)
    s.set_kdtree(tree)
    rng = np.random.default_rng(1)
    rays = np.zeros((4000, 8), np.float32)
    rays[:, :3] = rng.uniform(-0.9, 0.9, (4000, 3))
    d = rng.normal(size=(4000, 3))
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 6], rays[:, 7] = 1e-4, np.inf
    t0, p0 = O.trace_closest_brute(s.desc, rays)
    t1, _, _, p1 = O.trace_closest(s.desc, rays)
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(t1, t0)


def test_set_kdtree_rejects_bad_indices():
    s = mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {"width": 16, "height": 16, "spp": 1})
    n = s.prim_bounds().shape[0]
    bad = dict(nodes=np.array([[0x80000000, 1]], np.uint32), indices=np.array([n], np.uint32),
               aabb_min=np.zeros(3, np.float32), aabb_max=np.ones(3, np.float32), max_depth=0)
    with pytest.raises(RuntimeError, match="out of range"):
        s.set_kdtree(bad)


@pytest.mark.parametrize("nodes,n_idx,max_depth,msg", [
    ([[0x80000000, 2]], 1, 0, "range outside"),                          # leaf end past the index list
    ([[0x80000002, 1]], 1, 0, "range outside"),                          # leaf start > end
    ([[0 | (5 << 2), 0], [0x80000000, 0], [0x80000000, 0]], 0, 1, "children outside"),   # left child past the end
    ([[1 | (0 << 2), 0]], 0, 1, "children outside"),                     # left == self (cycle)
    ([[3 | (1 << 2), 0], [0x80000000, 0], [0x80000000, 0]], 0, 1, "not an inner node"),   # axis 3
    ([[0x40000000 | (1 << 2), 0], [0x80000000, 0], [0x80000000, 0]], 0, 1, "not an inner node"),   # indirection
    ([[0 | (1 << 2), 0], [0x80000000, 0], [0x80000000, 0]], 0, 0, "max_depth"),
    # two inner nodes sharing one child pair: node 3 reached twice
    ([[0 | (1 << 2), 0], [0 | (2 << 2), 0], [0 | (1 << 2), 0], [0x80000000, 0], [0x80000000, 0]], 0, 3, "twice"),
])
def test_set_kdtree_rejects_malformed_nodes(nodes, n_idx, max_depth, msg):
    """mtsh_scene_set_kdtree walks the node structure before the tree can
    reach the device traversal (it used to check indices only)."""
    s = mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {"width": 16, "height": 16, "spp": 1})
    bad = dict(nodes=np.array(nodes, np.uint32), indices=np.zeros(n_idx, np.uint32),
               aabb_min=np.zeros(3, np.float32), aabb_max=np.ones(3, np.float32), max_depth=max_depth)
    with pytest.raises(RuntimeError, match=msg):
        s.set_kdtree(bad)
