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
