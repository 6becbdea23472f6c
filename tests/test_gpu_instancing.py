"""Two-level instancing on the GPU (instance.cpp:115-160,
shapegroup.cpp:94-101) against the oracle's restatement on the same
two-level scene: closest hits bit-identical (same primitive => same t, u,
v), shadow occlusion equal, renders within the image L1 bar; the C4 tile
shares still sum to the frame."""
import os

import numpy as np
import pytest

import mtsg
from conftest import SCENES
from oracle import pyoracle as O
from test_gpu_parity import check_render, compare_closest, render_pair
from test_instancing import chords

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def inst_scene():
    s = mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 160, "height": 90, "spp": 4}, instancing="two-level")
    g = mtsg.GPUScene(s, 0)
    yield s, g
    g.close()


def test_two_level_closest_hits(inst_scene):
    s, g = inst_scene
    assert compare_closest(s, g, chords(200000, 7)) > 0.2


def test_two_level_closest_hits_from_surfaces(inst_scene):
    # secondary-ray-like queries: origins on the ground and inside the grid,
    # adaptive epsilon (mint = Epsilon)
    rng = np.random.default_rng(8)
    n = 100000
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0] = rng.uniform(-3.2, 3.2, n)
    rays[:, 1] = rng.uniform(0.0, 1.2, n)
    rays[:, 2] = rng.uniform(-2.0, 2.0, n)
    d = rng.normal(size=(n, 3))
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 6] = 1e-4
    rays[:, 7] = np.inf
    s, g = inst_scene
    assert compare_closest(s, g, rays) > 0.3


def test_two_level_shadow_rays(inst_scene):
    s, g = inst_scene
    rays = chords(100000, 9)
    rays[:, 7] = np.random.default_rng(10).uniform(0.1, 5.0, len(rays))
    o0 = O.trace_shadow(s.desc, rays)
    o1 = g.trace_shadow(rays)
    assert (o0 != o1).mean() < 1e-4
    assert o0.mean() > 0.05


def test_two_level_render_parity(inst_scene):
    s, g = inst_scene
    _, c, gi = render_pair(s, g)
    check_render(c, gi)
    for over in ({"max_depth": 2}, {"rr_depth": 1, "max_depth": 12}, {"strict_normals": 1}):
        _, c, gi = render_pair(s, g, **over)
        check_render(c, gi)


def test_two_level_c4_shares(inst_scene):
    s, g = inst_scene
    b = s.border
    full = g.render(s.params(), b)
    acc = sum(g.render(s.params(tile_stride=4, tile_offset=r), b) for r in range(4))
    np.testing.assert_allclose(acc, full, rtol=2e-5, atol=2e-6)


def test_two_level_c3_full_frame_parity():
    scene = mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 1280, "height": 720, "spp": 2},
                       instancing="two-level")
    g = mtsg.GPUScene(scene, 0)
    _, c, gi = render_pair(scene, g)
    g.close()
    l1, mean = check_render(c, gi)
    print(f"C3 two-level 1280x720x2spp: per-pixel L1 {l1:.3e}, mean {mean:.4f}")


def _rot_y(deg):
    a = np.radians(deg)
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def test_two_level_coplanar_tie_policy():
    """Exact ties inside instances (scenes/cbox_inst.xml: a group of three
    touching cubes, so two pairs of its faces coincide).  Rays from inside a
    cube through a shared face meet two triangles of the group at exactly
    the same distance.  Mitsuba resolves that in the group's own
    ShapeKDTree, with that traversal's own 8-entry mailbox (instance.cpp:
    115-130, sahkdtree3.h:250-290); the GPU flags the tie in its two-level
    iteration and traces the ray again with a literal two-level Havran
    (kernels.h tie_retrace_i), so the winner, t and u must be the oracle's
    bit for bit -- and a render of the scene is at parity."""
    scene = mtsg.Scene(os.path.join(SCENES, "cbox_inst.xml"), {"width": 48, "height": 48, "spp": 8},
                       instancing="two-level")
    rng = np.random.default_rng(23)
    # (group-space cube centre, main direction): through x = 0.25 and y = 0.25
    cases = [((0, 0, 0), (1, 0, 0)), ((0.5, 0, 0), (-1, 0, 0)), ((0, 0, 0), (0, 1, 0)), ((0, 0.5, 0), (0, -1, 0))]
    inst = [(np.eye(3), np.array([-0.5, -0.75, -0.25])), (_rot_y(-25), np.array([0.125, -0.75, 0.375]))]
    rays, planes = [], []
    n = 3000
    for R, off in inst:
        for c, dmain in cases:
            og = np.asarray(c) + rng.uniform(-0.2, 0.2, (n, 3))
            dg = np.asarray(dmain, float) + rng.normal(0, 0.15, (n, 3))
            dg /= np.linalg.norm(dg, axis=1, keepdims=True)
            r = np.zeros((n, 8), np.float32)
            r[:, :3] = og @ R.T + off
            r[:, 3:6] = dg @ R.T
            r[:, 6], r[:, 7] = 1e-4, np.inf
            rays.append(r)
            planes.append((R, off, 0 if dmain[0] else 1))
    n_cop = len(rays) * n
    m = 60000
    r = np.zeros((m, 8), np.float32)
    r[:, :3] = rng.uniform(-0.95, 0.95, (m, 3))
    d = rng.normal(size=(m, 3))
    r[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    r[:, 6], r[:, 7] = 1e-4, np.inf
    allr = np.concatenate(rays + [r])
    g = mtsg.GPUScene(scene, 0)
    try:
        t0, u0, v0, p0 = O.trace_closest(scene.desc, allr)
        t1, u1, v1, p1 = g.trace_closest(allr)
        # the designed rays do end on the coincident faces (group-space
        # coordinate 0.25 on the crossed axis)
        on = 0
        for k, (R, off, ax) in enumerate(planes):
            sl = slice(k * n, (k + 1) * n)
            hp = allr[sl, :3] + allr[sl, 3:6] * t0[sl, None]
            gp = (hp - off) @ R
            on += int((np.abs(gp[:, ax] - 0.25) < 1e-5).sum())
        assert on > 0.5 * n_cop, on
        hit = p0 != 0xFFFFFFFF
        np.testing.assert_array_equal(p1, p0)
        np.testing.assert_array_equal(t1, t0)
        np.testing.assert_array_equal(u1[hit], u0[hit])
        np.testing.assert_array_equal(v1[hit], v0[hit])
        _, c, gi = render_pair(scene, g)
        check_render(c, gi)
    finally:
        g.close()


SMALL_FAR_XML = """<?xml version="1.0"?>
<scene version="0.5.0">
  <sensor type="perspective"><transform name="toWorld"><lookat origin="0, 0, 3" target="0, 0, 0" up="0, 1, 0"/></transform>
    <film type="hdrfilm"><integer name="width" value="8"/><integer name="height" value="8"/></film></sensor>
  <shape type="shapegroup" id="g"><shape type="cube"><bsdf type="diffuse"/></shape></shape>
  <shape type="instance"><ref id="g"/><transform name="toWorld"><rotate y="1" angle="{rot}"/><scale value="{s}"/></transform></shape>
  <shape type="rectangle"><transform name="toWorld"><translate z="-5"/></transform>
    <emitter type="area"><rgb name="radiance" value="1"/></emitter></shape>
</scene>
"""


def _far_rays(size, dist, n=200000):
    """Rays from ~dist away aimed at points on and just outside the faces and
    edges of the rotated cube instance of SMALL_FAR_XML (world space)."""
    rng = np.random.default_rng(int(dist))
    q = rng.uniform(-1, 1, (n, 3))
    k = rng.integers(0, 3, n)
    q[np.arange(n), k] = np.sign(q[np.arange(n), k])
    edge = rng.random(n) < 0.5
    k2 = (k + 1) % 3
    q[edge, k2[edge]] = np.sign(q[edge, k2[edge]])
    q *= 1 + rng.uniform(-1e-5, 1e-5, (n, 1))
    c, sn = np.cos(np.radians(27.0)), np.sin(np.radians(27.0))
    w = np.stack([c * q[:, 0] + sn * q[:, 2], q[:, 1], -sn * q[:, 0] + c * q[:, 2]], 1) * size
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = w - d * dist
    rays[:, 3:6] = d
    rays[:, 6] = 1e-4
    rays[:, 7] = np.inf
    return rays


def _far_scene(tmp_path, size):
    p = tmp_path / "far.xml"
    p.write_text(SMALL_FAR_XML.format(rot=27.0, s=size))
    return mtsg.Scene(str(p), instancing="two-level")


def test_small_instance_seen_from_far_away(tmp_path):
    """a small instance at the origin (its world-box margin ~1e-4 of
    its size) hit by rays from 5e4 its size away, aimed at points on and just
    outside its faces and edges: hit/miss, primitive, t, u and v equal the
    oracle's two-level traversal for every ray."""
    s = _far_scene(tmp_path, 2e-3)
    g = mtsg.GPUScene(s, 0)
    rays = _far_rays(2e-3, 100.0)
    t0, u0, v0, p0 = O.trace_closest(s.desc, rays)
    t1, u1, v1, p1 = g.trace_closest(rays)
    g.close()
    hit0, hit1 = p0 != 0xFFFFFFFF, p1 != 0xFFFFFFFF
    assert hit0.mean() > 0.2, hit0.mean()
    assert np.array_equal(hit0, hit1), f"{(hit0 != hit1).sum()} rays disagree on hit/miss"
    same = p0 == p1
    assert same[hit0].mean() > 0.999
    np.testing.assert_array_equal(t1[same & hit0], t0[same & hit0])
    np.testing.assert_array_equal(u1[same & hit0], u0[same & hit0])


def test_instance_prefilter_drops_only_rejected_entries(tmp_path):
    """The world-box prefilter (kernels.h inst_box, widened by the instance's
    size and by 2^-20 of the ray origin's magnitude) against the same traversal
    without it (mtsg_test_knobs.no_instance_prefilter): every ray's hit is
    identical, also where the origin is 1e6 times the instance's size away.
    (There, at group-space magnitudes of 1e6, Mitsuba's own Havran traversal --
    the oracle -- loses some of the hits brute force finds: its entry/exit points
    o + t d carry ulp(|o|) errors of a few percent of the object; the t-interval
    traversal loses fewer, so the oracle is no bit-level reference at that
    scale: DESIGN.md §5.)"""
    for size, dist in ((2e-3, 100.0), (1e-3, 1000.0)):
        s = _far_scene(tmp_path, size)
        rays = _far_rays(size, dist)
        g = mtsg.GPUScene(s, 0)
        t1, u1, v1, p1 = g.trace_closest(rays)
        g.set_test_knobs(no_instance_prefilter=True)
        t2, u2, v2, p2 = g.trace_closest(rays)
        g.close()
        assert (p1 != 0xFFFFFFFF).mean() > 0.2
        np.testing.assert_array_equal(p1, p2)
        np.testing.assert_array_equal(t1, t2)
        np.testing.assert_array_equal(u1, u2)
        np.testing.assert_array_equal(v1, v2)
