"""Tail mode (k_finish): once a bounce starts with few paths, one persistent
launch carries them through their remaining bounces instead of a trace and a
shade launch per bounce.  It runs MIPathTracer::Li's loop body
(src/integrators/path/path.cpp:119-294) with the same arithmetic in the same
order per path, so every sample's radiance must be bit-identical to the
per-bounce kernels wherever the switch happens -- here from bounce 1 on
(threshold above any path count) against tail mode off."""
import os

import numpy as np
import pytest

import mtsg
from conftest import SCENES

pytestmark = pytest.mark.gpu

ALWAYS = 0xFFFFFFFF


def samples(scene, finish_paths, **over):
    g = mtsg.GPUScene(scene, 0)
    try:
        g.set_finish_paths(finish_paths)
        return g.render_samples(scene.params(**over)), g.stats()
    finally:
        g.close()


@pytest.mark.parametrize("name,defs", [
    ("bunny15.xml", {"width": 160, "height": 90, "spp": 4}),            # C3 scene, roughconductor
    ("cbox.xml", {"width": 64, "height": 48, "spp": 8}),                # diffuse, infinite depth
    ("cbox_materials.xml", {"width": 48, "height": 48, "spp": 8}),      # plastic, conductor, twosided
    ("env_glass.xml", {"width": 64, "height": 36, "spp": 4, "maxDepth": 16}),   # envmap + dielectric
])
def test_tail_mode_is_bit_identical(name, defs):
    scene = mtsg.Scene(os.path.join(SCENES, name), defs)
    ref, st0 = samples(scene, 0)
    out, st1 = samples(scene, ALWAYS)
    assert st0.launches_finish == 0
    assert st1.launches_finish == 1 and st1.paths_finish > 0
    assert np.array_equal(ref, out), f"{np.count_nonzero((ref != out).any(-1))} samples differ"


def test_tail_mode_with_qmc_samplers(tmp_path):
    # the sampler's dimension state travels through the in-place path records
    from test_gpu_samplers import SAMPLERS
    from test_samplers import sampler_scene
    for smp in ("halton", "hammersley", "ldsampler", "sobol"):
        s = sampler_scene(tmp_path, SAMPLERS[smp], width=32, height=32, spp=8)
        ref, _ = samples(s, 0)
        out, st = samples(s, ALWAYS)
        assert st.launches_finish == 1
        assert np.array_equal(ref, out), smp


def test_tail_mode_threshold_switches_late():
    # a threshold between the bounce sizes switches mid-frame; the film is unchanged
    scene = mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 160, "height": 90, "spp": 4})
    ref, _ = samples(scene, 0)
    out, st = samples(scene, 20000)
    assert st.launches_finish == 1 and 0 < st.paths_finish < 20000
    assert np.array_equal(ref, out)


@pytest.mark.parametrize("name,defs", [
    ("bunny15.xml", {"width": 160, "height": 90, "spp": 4}),
    ("bunny15.xml", {"width": 96, "height": 54, "spp": 4, "maxDepth": 16}),
])
def test_tail_mode_two_level_is_bit_identical(name, defs):
    # two-level instancing: the tail kernel switches levels per lane like
    # k_trace_s<.., true>, with the instance of each hit for the shading
    scene = mtsg.Scene(os.path.join(SCENES, name), defs, instancing="two-level")
    ref, st0 = samples(scene, 0)
    out, st1 = samples(scene, ALWAYS)
    assert st0.launches_finish == 0
    assert st1.launches_finish == 1 and st1.paths_finish > 0
    assert np.array_equal(ref, out), f"{np.count_nonzero((ref != out).any(-1))} samples differ"
