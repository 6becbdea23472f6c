"""GPU parity of the samplers: the device draws equal the
oracle's bit for bit (tests/test_samplers.py pins the oracle), and renders
with each sampler match the oracle's renders (same bar as test_gpu_parity)."""
import numpy as np
import pytest

import mtsg
from oracle import pyoracle as O
from test_samplers import sampler_scene
from test_gpu_parity import render_pair, check_render

pytestmark = pytest.mark.gpu

SAMPLERS = {
    "independent": '<sampler type="independent"><integer name="sampleCount" value="$spp"/></sampler>',
    "halton": '<sampler type="halton"><integer name="sampleCount" value="$spp"/></sampler>',
    "halton_plain": '<sampler type="halton"><integer name="scramble" value="0"/>'
                    '<integer name="sampleCount" value="$spp"/></sampler>',
    "halton_random": '<sampler type="halton"><integer name="scramble" value="7"/>'
                     '<integer name="sampleCount" value="$spp"/></sampler>',
    "hammersley": '<sampler type="hammersley"><integer name="sampleCount" value="$spp"/></sampler>',
    "ldsampler": '<sampler type="ldsampler"><integer name="sampleCount" value="$spp"/></sampler>',
    "sobol": '<sampler type="sobol"><integer name="sampleCount" value="$spp"/></sampler>',
    "sobol_scrambled": '<sampler type="sobol"><integer name="scramble" value="9"/>'
                       '<integer name="sampleCount" value="$spp"/></sampler>',
}


@pytest.mark.parametrize("name", sorted(SAMPLERS))
def test_sampler_draws_match_oracle(tmp_path, name):
    sc = sampler_scene(tmp_path, SAMPLERS[name], width=48, height=40, spp=16)
    g = mtsg.GPUScene(sc, 0)
    p = sc.params(seed=5)
    kinds = [2, 2, 2, 1, 2, 2, 1, 2, 2, 1, 2, 2, 1, 1, 2]
    for (x, y) in ((0, 0), (17, 9), (47, 39)):
        for s in (0, 3, 15):
            want = O.sampler_draws(sc.desc, p, x, y, s, kinds)
            got = g.sampler_draws(p, x, y, s, kinds)
            np.testing.assert_array_equal(got, want, err_msg=f"{name} pixel ({x},{y}) sample {s}")
    g.close()


@pytest.mark.parametrize("name,msg", [("halton", "prime number table"), ("sobol", "direction number table")])
def test_device_dimension_limit(tmp_path, name, msg):
    sc = sampler_scene(tmp_path, SAMPLERS[name], width=8, height=8, spp=4)
    g = mtsg.GPUScene(sc, 0)
    g.sampler_draws(sc.params(), 0, 0, 0, [1] * 1024)
    with pytest.raises(RuntimeError, match=msg):
        g.sampler_draws(sc.params(), 0, 0, 0, [1] * 1025)
    g.close()


@pytest.mark.parametrize("name", ["halton", "hammersley", "ldsampler", "sobol", "sobol_scrambled"])
def test_render_parity_per_sampler(tmp_path, name):
    sc = sampler_scene(tmp_path, SAMPLERS[name], width=64, height=48, spp=8)
    g = mtsg.GPUScene(sc, 0)
    for over in ({}, {"max_depth": 3, "tile_x": 5, "tile_y": 7, "tile_w": 37, "tile_h": 19}):
        _, c, gi = render_pair(sc, g, **over)
        check_render(c, gi)
    g.close()


def test_ldsampler_rejects_non_power_of_two_counts(tmp_path):
    sc = sampler_scene(tmp_path, SAMPLERS["ldsampler"], width=16, height=16, spp=8)
    g = mtsg.GPUScene(sc, 0)
    with pytest.raises(RuntimeError):
        g.render(sc.params(spp=6), sc.border)
    g.close()
