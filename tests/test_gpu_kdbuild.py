"""The device-side SAH kd-tree build (mtsg_kd_build).

The GPU tree is a different tree from the host's (binned instead of exact
SAH, no retraction of bad splits), so parity is asserted on what a tree must answer:
- structure: Mitsuba's KDNode encoding, every live primitive referenced,
  leaf ranges inside the index list, depth within maxDepth;
- closest hits: the oracle's Havran traversal over the device-built tree
  against brute force over every primitive (same primitive except exact
  distance ties, bit-identical t), and the GPU traversal over it against the
  GPU traversal over the host-built tree;
- renders: the GPU with the device-built tree against the oracle with the
  host-built tree (counter mode, per-pixel L1 < 1e-3 of the mean);
- build time on the C3 scene, against the host build (reported, and the
  device build must be the faster one)."""
import os

import numpy as np
import pytest

import mtsg
from oracle import pyoracle as O
from conftest import SCENES
from test_gpu_parity import check_render, random_rays, render_pair

pytestmark = pytest.mark.gpu


def walk(tree, n_prims, bounds):
    nodes, idx = tree["nodes"], tree["indices"]
    seen = np.zeros(n_prims, bool)
    stack = [(0, 0)]
    deepest = 0
    while stack:
        i, d = stack.pop()
        deepest = max(deepest, d)
        c, data = int(nodes[i, 0]), int(nodes[i, 1])
        if c & 0x80000000:
            s, e = c & 0x7FFFFFFF, data
            assert s <= e <= idx.size
            seen[idx[s:e]] = True
            assert (np.diff(idx[s:e].astype(np.int64)) > 0).all()   # sorted, no duplicates
        else:
            left = i + ((c & ~(3 | 0x40000000)) >> 2)
            assert i < left < nodes.shape[0] - 1
            stack += [(left, d + 1), (left + 1, d + 1)]
    live = (bounds[:, :3] <= bounds[:, 3:]).all(1)
    assert seen[live].all() and not seen[~live].any()
    assert deepest == tree["max_depth"]
    return deepest


@pytest.mark.parametrize("name,defs", [("cbox.xml", {}), ("cbox_textured.xml", {}), ("env_glass.xml", {})])
def test_structure_and_brute_force_hits(name, defs):
    s = mtsg.Scene(os.path.join(SCENES, name), dict(defs, width=32, height=24, spp=1))
    b = s.prim_bounds()
    tree = mtsg.kd_build(s, b)
    walk(tree, b.shape[0], b)
    s.set_kdtree(tree)
    lo, hi = tree["aabb_min"], tree["aabb_max"]
    rays = random_rays(20000, lo + 0.2 * (hi - lo), hi - 0.2 * (hi - lo), seed=3)
    t0, p0 = O.trace_closest_brute(s.desc, rays)
    t1, _, _, p1 = O.trace_closest(s.desc, rays)
    hit0, hit1 = p0 != 0xFFFFFFFF, p1 != 0xFFFFFFFF
    # exact: a reference lost by the build (e.g. a clipped bound rounded
    # across a split plane) shows up here as a miss
    np.testing.assert_array_equal(hit1, hit0)
    both = hit0 & hit1
    same = both & (p0 == p1)
    np.testing.assert_array_equal(t1[same], t0[same])
    # another primitive only on ties: coplanar triangles sharing the hit point
    # (brute force reports the lowest index, Havran the first in leaf order)
    diff = both & (p0 != p1)
    np.testing.assert_allclose(t1[diff], t0[diff], rtol=1e-6)
    assert same.sum() >= 0.995 * both.sum()


@pytest.fixture(scope="module")
def c3():
    host = mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 160, "height": 90, "spp": 4})
    dev = mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 160, "height": 90, "spp": 4})
    b = dev.prim_bounds()
    mtsg.kd_build(dev, b)   # warm-up (module load, first allocations)
    tree = mtsg.kd_build(dev, b)
    dev.set_kdtree(tree)
    return host, dev, tree, b


def test_c3_device_tree(c3):
    host, dev, tree, b = c3
    depth = walk(tree, b.shape[0], b)
    print(f"C3 device build: {tree['ms']:.1f} ms, {tree['nodes'].shape[0]} nodes, {tree['indices'].size} refs, "
          f"{tree['leaves']} leaves, depth {depth}; host build {host.info.kd_build_seconds * 1e3:.1f} ms, "
          f"{host.info.kd_nodes} nodes, {host.info.kd_indices} refs")
    assert tree["ms"] < host.info.kd_build_seconds * 1e3
    gh, gd = mtsg.GPUScene(host, 0), mtsg.GPUScene(dev, 0)
    lo, hi = tree["aabb_min"], tree["aabb_max"]
    rays = random_rays(200000, lo + 0.1 * (hi - lo), hi - 0.1 * (hi - lo), seed=11)
    th, _, _, ph = gh.trace_closest(rays)
    td, _, _, pd = gd.trace_closest(rays)
    hh, hd = ph != 0xFFFFFFFF, pd != 0xFFFFFFFF
    np.testing.assert_array_equal(hd, hh)
    both = hh & hd
    same = both & (ph == pd)
    assert same.sum() >= 0.999 * both.sum()
    np.testing.assert_array_equal(td[same], th[same])
    # a render through the device-built tree against the oracle on the host-built one
    _, c, _ = render_pair(host, gh)
    gi = gd.render(dev.params(), dev.border)
    check_render(c, gi)
    gh.close()
    gd.close()


def leaf_sets(tree):
    """{node index: the leaf's primitive indices} of a tree dict"""
    nodes, idx = tree["nodes"], tree["indices"]
    out = {}
    for i in range(nodes.shape[0]):
        c, d = int(nodes[i, 0]), int(nodes[i, 1])
        if c & 0x80000000:
            out[i] = tuple(idx[c & 0x7FFFFFFF:d].tolist())
    return out


def test_refit_unchanged_geometry_gives_the_same_leaves():
    """mtsg_kd_refit over the geometry the tree was built on: the nodes keep
    their words and every leaf gets back its primitives (the build's
    classification and clipping; retracted leaves hold the union of their
    former subtrees), except a primitive lying flat in a split plane: the
    build's exact sweep chose its side, which the KDNode encoding does not
    record, and the refit puts it on the left (both are exact).  The trees
    answer every query identically."""
    s = mtsg.Scene(os.path.join(SCENES, "cbox_glass.xml"), {"width": 32, "height": 24, "spp": 1})
    b = s.prim_bounds()
    tree = mtsg.kd_build(s, b)
    re = mtsg.kd_refit(s, tree, b)
    walk(re, b.shape[0], b)
    leaf = (tree["nodes"][:, 0] & 0x80000000) != 0
    np.testing.assert_array_equal((re["nodes"][:, 0] & 0x80000000) != 0, leaf)
    np.testing.assert_array_equal(re["nodes"][~leaf], tree["nodes"][~leaf])
    flat = (b[:, :3] == b[:, 3:]).any(1)
    a0, a1 = leaf_sets(tree), leaf_sets(re)
    moved = 0
    for i in a0:
        d = set(a0[i]) ^ set(a1[i])
        assert all(flat[k] for k in d), (i, d)
        moved += len(d)
    print(f"refit of cbox_glass's device tree: {moved} of {tree['indices'].size} references of planar primitives changed sides")
    rays = random_rays(20000, -0.95, 0.95, seed=6)
    s.set_kdtree(tree)
    t0, u0, v0, p0 = O.trace_closest(s.desc, rays)
    s.set_kdtree(re)
    t1, u1, v1, p1 = O.trace_closest(s.desc, rays)
    np.testing.assert_array_equal(t1, t0)
    hit = p0 != 0xFFFFFFFF
    same = p0 == p1
    assert same.mean() > 0.999   # another primitive only on exact ties
    np.testing.assert_array_equal(u1[same & hit], u0[same & hit])


def test_refit_moved_geometry_answers_exactly():
    """The tree of the Cornell box with the glass box on its default place,
    refit after the box moved 0.5 up (the same XML, -D glassY): the refit tree
    must answer every closest-hit query as brute force over the moved scene
    does (the Havran traversal of the oracle over it), and the GPU over it must
    render the moved scene at parity."""
    a = mtsg.Scene(os.path.join(SCENES, "cbox_glass.xml"), {"width": 32, "height": 24, "spp": 1})
    m = mtsg.Scene(os.path.join(SCENES, "cbox_glass.xml"), {"width": 32, "height": 24, "spp": 2, "glassY": -0.199})
    ba, bm = a.prim_bounds(), m.prim_bounds()
    assert ba.shape == bm.shape and not np.array_equal(ba, bm)
    tree = mtsg.kd_build(a, ba)
    re = mtsg.kd_refit(m, tree, bm)
    walk(re, bm.shape[0], bm)
    m.set_kdtree(re)
    rays = random_rays(20000, -0.95, 0.95, seed=5)
    t0, p0 = O.trace_closest_brute(m.desc, rays)
    t1, _, _, p1 = O.trace_closest(m.desc, rays)
    hit0, hit1 = p0 != 0xFFFFFFFF, p1 != 0xFFFFFFFF
    np.testing.assert_array_equal(hit1, hit0)
    # exactness: every hit at brute force's distance, bit for bit (a primitive
    # the refit dropped from a leaf would leave a farther hit: another t); only
    # the primitive may differ, and only where two meet the ray at that t
    np.testing.assert_array_equal(t1[hit0], t0[hit0])
    same = hit0 & (p0 == p1)
    assert same.sum() >= 0.995 * hit0.sum()
    g = mtsg.GPUScene(m, 0)
    try:
        t2, _, _, p2 = g.trace_closest(rays)
        np.testing.assert_array_equal(p2, p1)
        np.testing.assert_array_equal(t2, t1)
        _, c, gi = render_pair(m, g)
        check_render(c, gi)
    finally:
        g.close()


def test_c3_refit_time(c3):
    """Refit of the C3 device tree over its own geometry: the time a
    per-frame update of 1M triangles costs against the full build."""
    host, dev, tree, b = c3
    mtsg.kd_refit(dev, tree, b)   # warm-up
    re = mtsg.kd_refit(dev, tree, b)
    walk(re, b.shape[0], b)
    print(f"C3 refit: {re['ms']:.1f} ms (device build {tree['ms']:.1f} ms), {re['indices'].size} refs "
          f"(build {tree['indices'].size})")
    assert re["indices"].size == tree["indices"].size
    assert re["ms"] < tree["ms"]
