"""Two-level instancing on the host and in the oracle:
Mitsuba's `instance` / `shapegroup` structure (src/shapes/instance.cpp:107-160,
src/shapes/shapegroup.cpp:94-101) -- one group-space kd-tree, instances as
primitives of the top-level tree, rays transformed per instance visit.  The
flattened variant (world-space copies of every instance's triangles) is the
same geometry, so both must find the same closest surfaces."""
import os

import numpy as np
import pytest

import mtsg
from conftest import SCENES
from oracle import pyoracle as O


@pytest.fixture(scope="module")
def two_level():
    return mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 96, "height": 54, "spp": 2},
                      instancing="two-level")


@pytest.fixture(scope="module")
def flat():
    return mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 96, "height": 54, "spp": 2})


def chords(n, seed):
    rng = np.random.default_rng(seed)
    c = np.array([0.0, 0.45, 0.0])

    def sph(k):
        v = rng.normal(size=(k, 3))
        return v / np.linalg.norm(v, axis=1, keepdims=True)
    a = c + 3.2 * sph(n)
    b = c + 3.2 * sph(n)
    d = (b - a) / np.linalg.norm(b - a, axis=1, keepdims=True)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = a
    rays[:, 3:6] = d
    rays[:, 6] = 0.0
    rays[:, 7] = np.inf
    return rays


def test_two_level_scene_structure(two_level, flat):
    # 15 instance primitives replace 15 x 69,451 world-space triangles in the top-level tree
    assert two_level.info.n_triangles == 69451
    assert flat.info.n_triangles == 15 * 69451
    assert two_level.info.kd_indices < 200   # instances + ground + light only


def test_two_level_traversal_matches_brute_force(two_level):
    rays = chords(4000, 3)
    t, u, v, prim = O.trace_closest(two_level.desc, rays)
    tb, pb = O.trace_closest_brute(two_level.desc, rays)
    hit = prim != 0xFFFFFFFF
    assert hit.mean() > 0.2
    np.testing.assert_array_equal(hit, pb != 0xFFFFFFFF)
    np.testing.assert_array_equal(t[hit], tb[hit])
    assert (prim[hit] == pb[hit]).mean() > 0.999


def test_two_level_hits_the_flattened_surfaces(two_level, flat):
    rays = chords(20000, 4)
    t2, _, _, p2 = O.trace_closest(two_level.desc, rays)
    tf, _, _, pf = O.trace_closest(flat.desc, rays)
    h2, hf = p2 != 0xFFFFFFFF, pf != 0xFFFFFFFF
    assert (h2 != hf).mean() < 1e-3
    both = h2 & hf
    # same triangle of the group (flattened index = instance * 69451 + group index)
    assert ((pf[both] % 69451) == (p2[both] % 69451)).mean() > 0.995
    np.testing.assert_allclose(t2[both], tf[both], rtol=2e-4, atol=1e-5)


def test_two_level_shadow_rays(two_level, flat):
    rays = chords(20000, 5)
    rays[:, 7] = np.random.default_rng(6).uniform(0.1, 5.0, len(rays))
    o2 = O.trace_shadow(two_level.desc, rays)
    of = O.trace_shadow(flat.desc, rays)
    assert (o2 != of).mean() < 1e-3
    assert o2.mean() > 0.05


def test_two_level_render_matches_flattened_statistically(two_level, flat):
    p = two_level.params(spp=8)
    b = two_level.border
    i2, _ = O.render(two_level.desc, p, b, rng=O.RNG_COUNTER)
    i1, _ = O.render(flat.desc, p, b, rng=O.RNG_COUNTER)
    r2, r1 = mtsg.develop(i2), mtsg.develop(i1)
    # identical random numbers, geometry equal up to float rounding: paths
    # diverge only where a rounding difference changes a decision
    assert abs(r2.mean() - r1.mean()) < 0.01 * r1.mean()
    assert (np.abs(r2 - r1) > 1e-3).mean() < 0.05


def test_instancing_errors(tmp_path):
    src = open(os.path.join(SCENES, "bunny15.xml")).read()
    bad = src.replace('<ref id="bunny"/>\n\t\t<transform name="toWorld">\n\t\t\t<rotate y="1" angle="0.0000"/>',
                      '<transform name="toWorld">\n\t\t\t<rotate y="1" angle="0.0000"/>', 1)
    p = tmp_path / "noref.xml"
    p.write_text(bad.replace('filename" value="bunny.ply', 'filename" value="' + os.path.join(SCENES, "bunny.ply")))
    for mode in ("flatten", "two-level"):
        with pytest.raises(RuntimeError, match="shapegroup"):
            mtsg.Scene(str(p), {"width": 8, "height": 8, "spp": 1}, instancing=mode)
    with pytest.raises(ValueError):
        mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), instancing="deep")
