"""Degenerate ray queries through the device traversal (mtsg_trace_closest /
mtsg_trace_shadow -> k_trace_s) against the oracle's Havran restatement:
- axis-aligned directions and directions with one zero component (the
  scene-AABB slab test of spec_init takes its `d == 0` branch, aabb.h:308-338;
  the split-plane distance is +-inf or NaN, sahkdtree3.h:214-228);
- origins exactly on the scene bounds' faces, moving along the face (grazing)
  or inward;
- origins on primitive-bound planes, the candidate planes of the SAH build
  (gkdtree.h), so many lie exactly on split planes of the tree;
- empty and reversed intervals (mint >= maxt), which must miss;
over the flattened C3 scene, the Cornell box and the two-level C3 scene.
Same primitive => bit-identical t, u, v (compare_closest); occlusion equal."""
import os

import numpy as np
import pytest

import mtsg
from conftest import SCENES
from oracle import pyoracle as O
from test_gpu_parity import compare_closest

pytestmark = pytest.mark.gpu


def bounds(scene):
    b = scene.prim_bounds()
    live = (b[:, :3] <= b[:, 3:]).all(1)
    return b[live, :3].min(0).astype(np.float32), b[live, 3:].max(0).astype(np.float32)


def degenerate_rays(lo, hi, n, seed, planes=None):
    rng = np.random.default_rng(seed)
    rays = np.zeros((n, 8), np.float32)
    ext = hi - lo
    o = rng.uniform(lo + 0.05 * ext, hi - 0.05 * ext, (n, 3)).astype(np.float32)
    d = np.zeros((n, 3), np.float32)
    kind = rng.integers(0, 4, n)
    # 0: +-axis; 1: one zero component; 2: face origin moving along the face;
    # 3: face origin moving inward along the axis
    ax = rng.integers(0, 3, n)
    sgn = np.where(rng.random(n) < 0.5, -1.0, 1.0).astype(np.float32)
    idx = np.arange(n)
    m = kind == 0
    d[idx[m], ax[m]] = sgn[m]
    m = (kind == 1) | (kind == 2)
    v = rng.normal(size=(n, 3)).astype(np.float32)
    v[idx, ax] = 0.0
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    d[m] = v[m]
    m = (kind == 2) | (kind == 3)
    face = np.where(sgn > 0, lo[ax], hi[ax])   # the face the inward axis ray starts on
    o[idx[m], ax[m]] = face[m]
    m = kind == 3
    d[idx[m], ax[m]] = sgn[m]
    if planes is not None:   # a quarter of the origins on primitive-bound planes
        m = np.flatnonzero(rng.random(n) < 0.25)
        k = rng.integers(0, planes.shape[0], m.size)
        c = rng.integers(0, 6, m.size)
        o[m, c % 3] = planes[k, c]
    rays[:, 0:3] = o
    rays[:, 3:6] = d
    rays[:, 6] = 1e-4
    rays[:, 7] = np.inf
    return rays


def planes(scene):
    b = scene.prim_bounds()
    return b[(b[:, :3] <= b[:, 3:]).all(1)].astype(np.float32)


@pytest.fixture(scope="module", params=["cbox", "bunny15", "bunny15-two-level"])
def scene_pair(request):
    name = request.param
    inst = "two-level" if name.endswith("two-level") else "flatten"
    xml = "cbox.xml" if name == "cbox" else "bunny15.xml"
    s = mtsg.Scene(os.path.join(SCENES, xml), {"width": 32, "height": 24, "spp": 1}, instancing=inst)
    g = mtsg.GPUScene(s, 0)
    yield s, g
    g.close()


def test_degenerate_closest(scene_pair):
    s, g = scene_pair
    lo, hi = bounds(s)
    rays = degenerate_rays(lo, hi, 60000, 41, planes(s))
    assert compare_closest(s, g, rays) > 0.1


def test_degenerate_shadow(scene_pair):
    s, g = scene_pair
    lo, hi = bounds(s)
    rays = degenerate_rays(lo, hi, 60000, 43, planes(s))
    rays[:, 7] = np.random.default_rng(44).uniform(0.01, float((hi - lo).max()), len(rays))
    o0 = O.trace_shadow(s.desc, rays)
    o1 = g.trace_shadow(rays)
    assert (o0 != o1).mean() < 1e-4
    assert 0.01 < o1.mean() < 0.99


def test_empty_intervals_miss(scene_pair):
    s, g = scene_pair
    lo, hi = bounds(s)
    rays = degenerate_rays(lo, hi, 4096, 45)
    rays[:2048, 7] = rays[:2048, 6]          # mint == maxt
    rays[2048:, 6] = 5.0
    rays[2048:, 7] = 1.0                     # mint > maxt
    _, _, _, p = g.trace_closest(rays)
    assert (p == 0xFFFFFFFF).all()
    assert not g.trace_shadow(rays).any()
    _, _, _, p0 = O.trace_closest(s.desc, rays)
    assert (p0 == 0xFFFFFFFF).all()


def corner_rays(scene, n, seed):
    """Rays from and towards corners of primitive bounds: points where three
    candidate split planes of the SAH build meet, so the traversal crosses
    several split planes at exactly the same distance (the case a short
    stack can drop entries on, again and again, at one restart distance)."""
    rng = np.random.default_rng(seed)
    p = planes(scene)
    a = p[rng.integers(0, p.shape[0], n)]
    b = p[rng.integers(0, p.shape[0], n)]
    ca = np.where(rng.random((n, 3)) < 0.5, a[:, :3], a[:, 3:])
    cb = np.where(rng.random((n, 3)) < 0.5, b[:, :3], b[:, 3:])
    d = (cb - ca).astype(np.float64)
    ln = np.linalg.norm(d, axis=1)
    ok = ln > 1e-6
    d = (d[ok] / ln[ok, None]).astype(np.float32)
    rays = np.zeros((d.shape[0], 8), np.float32)
    # start behind the first corner so that the ray passes through it
    rays[:, 0:3] = ca[ok] - 0.25 * d
    rays[:, 3:6] = d
    rays[:, 6] = 1e-4
    rays[:, 7] = np.inf
    return rays


@pytest.mark.parametrize("name", ["cbox", "bunny15", "bunny15-two-level"])
def test_restart_guard_terminates_and_matches(name):
    """Every traversal stack cut to one entry (mtsg_set_test_knobs): far children
    are dropped at almost every second push, rays kd-restart many times, and
    rays through split-plane corners return to the same restart distance.
    Without the guard such rays live-lock (they reach the restart limit:
    MTSG_ERR_TRAVERSAL instead of a hang); with it (kernels.h kd_restart)
    every query terminates with the same closest-hit distances, bit for bit,
    as the full stacks give.  (Exact corner rays are a degenerate case of Mitsuba's
    traversal itself -- the oracle's Havran restatement and brute force
    disagree on ~1% of them -- so the reference here is the full-stack
    traversal; test_degenerate_closest compares that with the oracle.)"""
    inst = "two-level" if name.endswith("two-level") else "flatten"
    xml = "cbox.xml" if name == "cbox" else "bunny15.xml"
    s = mtsg.Scene(os.path.join(SCENES, xml), {"width": 32, "height": 24, "spp": 1}, instancing=inst)
    rays = np.concatenate([corner_rays(s, 30000, 51), degenerate_rays(*bounds(s), 20000, 52, planes(s))])
    sh = rays.copy()
    sh[:, 7] = np.random.default_rng(53).uniform(0.01, 4.0, len(sh))
    g = mtsg.GPUScene(s, 0)
    ref, ref_sh = g.trace_closest(rays), g.trace_shadow(sh)
    g.close()
    g = mtsg.GPUScene(s, 0)
    try:
        g.set_test_knobs(stack_cap=1, restart_guard=100000)   # guard off
        with pytest.raises(RuntimeError, match=r"\(-6\).*restart limit"):
            g.trace_closest(rays)
        g.set_test_knobs(stack_cap=1)
        got, got_sh = g.trace_closest(rays), g.trace_shadow(sh)
    finally:
        g.close()
    # the same hits at the same distances, bit for bit; where several
    # primitives meet the ray at exactly that distance (box corners) the
    # leaf visit order decides which one is reported, and a restart can
    # reach those leaves in another order
    np.testing.assert_array_equal(got[3] == 0xFFFFFFFF, ref[3] == 0xFFFFFFFF)
    same = got[3] == ref[3]
    assert same.mean() > 0.99
    for k in range(3):
        np.testing.assert_array_equal(got[k][same], ref[k][same])
    # a tie: another primitive through the same point (its own t rounding)
    np.testing.assert_allclose(got[0][~same], ref[0][~same], rtol=1e-6)
    np.testing.assert_array_equal(got_sh, ref_sh)


def test_restart_limit_fails_the_query():
    """A ray that reaches the restart limit ends with an error the caller
    sees (MTSG_ERR_TRAVERSAL), from the debug queries and from the render,
    instead of the kernel spinning: limit 0 makes the first restart fail."""
    s = mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 64, "height": 36, "spp": 1})
    g = mtsg.GPUScene(s, 0)
    try:
        g.set_test_knobs(stack_cap=1, restart_limit=0)
        with pytest.raises(RuntimeError, match=r"\(-6\).*restart limit"):
            g.trace_closest(corner_rays(s, 20000, 54))
        with pytest.raises(RuntimeError, match=r"\(-6\).*restart limit"):
            g.render(s.params(), s.border)
        # with the default limit the frame renders
        g.set_test_knobs(stack_cap=1)
        g.render(s.params(), s.border)
        g.set_test_knobs()
        g.render(s.params(), s.border)
    finally:
        g.close()


def test_restart_limit_of_shadow_rays_fails_the_render():
    """The limit applied to shadow rays only (limit_shadow_only):
    closest-hit rays traverse normally, and a shadow ray that reaches the limit
    still fails the render.  Shadow rays are traced in the next bounce's launch
    or in the final shadow launch after the last bounce; the error word is read
    after both (the final launch's errors were not read)."""
    s = mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 64, "height": 36, "spp": 1})
    g = mtsg.GPUScene(s, 0)
    try:
        g.set_test_knobs(stack_cap=1, restart_limit=0, limit_shadow_only=True)
        rays = corner_rays(s, 20000, 55)
        g.trace_closest(rays)   # closest-hit rays are not limited
        sh = rays.copy()
        sh[:, 7] = 1e30
        with pytest.raises(RuntimeError, match=r"\(-6\).*restart limit"):
            g.trace_shadow(sh)
        for depth in (2, 3, -1):
            with pytest.raises(RuntimeError, match=r"\(-6\).*restart limit"):
                g.render(s.params(max_depth=depth), s.border)
    finally:
        g.close()
