"""GPU renders of scenes handed over through the in-memory builder
(mtsh_scene_begin / _add_* / _finish): what the Mitsuba-side plugin renders
(INTEGRATION.md).  The builder's scene is byte-identical to the XML route's
(tests/test_scene_builder.py); here the device renders it, through
mtsg_render and through the multi-GPU job, against the oracle in counter
mode (identical random numbers per pixel / sample / dimension), per-pixel."""
import os

import numpy as np
import pytest

import mtsg
import scene_walker as W
from oracle import pyoracle as O
from conftest import SCENES

pytestmark = pytest.mark.gpu


def per_pixel(a, b):
    return np.abs(mtsg.develop(a) - mtsg.develop(b)).mean(axis=-1)


# the share of pixels above a per-pixel L1 of 1e-3 allowed: none (glibc's
# float algorithms on the device keep even the glass scene's long specular
# chains on the oracle's paths)
@pytest.mark.parametrize("xml,defines,instancing,tail", [
    ("bunny15.xml", {"width": 96, "height": 54, "spp": 8}, "flatten", 0.0),
    ("bunny15.xml", {"width": 96, "height": 54, "spp": 8}, "two-level", 0.0),
    ("env_glass.xml", {"width": 96, "height": 54, "spp": 8, "maxDepth": 16}, "flatten", 0.0),
])
def test_builder_scene_renders_at_oracle_parity(xml, defines, instancing, tail):
    scene = W.build(os.path.join(SCENES, xml), defines, instancing=instancing, meshes="world")
    params = scene.params()
    g = mtsg.GPUScene(scene, 0)
    img_g = g.render(params, scene.border)
    g.close()
    img_c, _ = O.render(scene.desc, params, scene.border, rng=O.RNG_COUNTER)
    pp = per_pixel(img_g, img_c)
    mean = float(mtsg.develop(img_c).mean())
    print(f"{xml} {instancing}: mean {mean:.4f}, per-pixel L1 mean {pp.mean():.2e} max {pp.max():.2e}")
    assert mean > 0
    assert pp.mean() < 1e-3 * mean
    assert (pp > 1e-3).mean() <= tail


def test_bsdf_define_through_the_builder_renders_on_the_gpu(tmp_path):
    """A -D on a BSDF parameter, as the plugin hands it over, rendered by the
    multi-GPU job: the image of the -D scene, not of the file's default."""
    from test_scene_builder import OVERRIDE_XML
    p = tmp_path / "cbox_params.xml"
    p.write_text(OVERRIDE_XML.replace("{bunny}", os.path.join(SCENES, "bunny.ply")))
    scene = W.build(str(p), {"wallR": "0.15", "alpha": "0.5", "lightR": "30"})
    params = scene.params()
    job = mtsg.PathJob(scene, 0)
    rc, img_g, _ = job.render(params, scene.border)
    job.close()
    assert rc == mtsg.MTSG_OK
    img_c, _ = O.render(scene.desc, params, scene.border, rng=O.RNG_COUNTER)
    assert per_pixel(img_g, img_c).max() < 1e-3
    stale = mtsg.Scene(str(p), {})
    img_s, _ = O.render(stale.desc, stale.params(), stale.border, rng=O.RNG_COUNTER)
    assert per_pixel(img_g, img_s).mean() > 1e-2 * float(mtsg.develop(img_s).mean())
