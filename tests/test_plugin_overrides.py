"""The plugin binding of INTEGRATION.md: Mitsuba loads the scene with the
user's -D map (mitsuba.cpp:168-174, scenehandler.cpp:211) and the plugin
hands the values it holds in memory -- film size, the sampler's sample count,
the integrator's parameters -- to mtsh_scene_load_overrides, because the
parameter map itself does not reach the plugin.  The result must be the scene
the -D map describes: same render parameters and camera, and (oracle,
counter RNG) the same image, bit for bit."""
import os

import numpy as np
import pytest

from conftest import SCENES


def overrides_for(width, height, spp, max_depth=None, rr_depth=5, strict=0, hide=0):
    import mtsg
    ov = mtsg.SceneOverrides()
    ov.mask = mtsg.MTSH_OVERRIDE_FILM_SIZE | mtsg.MTSH_OVERRIDE_SAMPLE_COUNT
    ov.film_width, ov.film_height, ov.sample_count = width, height, spp
    if max_depth is not None:
        ov.mask |= mtsg.MTSH_OVERRIDE_INTEGRATOR
        ov.max_depth, ov.rr_depth, ov.strict_normals, ov.hide_emitters = max_depth, rr_depth, strict, hide
    return ov


def same_params(a, b):
    for f in ("tile_x", "tile_y", "tile_w", "tile_h", "spp", "max_depth", "rr_depth", "strict_normals",
              "hide_emitters"):
        assert getattr(a, f) == getattr(b, f), f


@pytest.mark.parametrize("xml,defs,ov", [
    ("cbox.xml", {"width": 40, "height": 24, "spp": 3, "maxDepth": 4},
     dict(width=40, height=24, spp=3, max_depth=4)),
    ("bunny15.xml", {"width": 32, "height": 20, "spp": 2}, dict(width=32, height=20, spp=2)),
])
def test_overrides_equal_defines(xml, defs, ov):
    import mtsg
    from oracle import pyoracle as O
    by_defines = mtsg.Scene(os.path.join(SCENES, xml), defs)
    by_plugin = mtsg.Scene(os.path.join(SCENES, xml), {}, overrides=overrides_for(**ov))
    pd, pp = by_defines.params(), by_plugin.params()
    same_params(pd, pp)
    assert (by_plugin.info.film_w, by_plugin.info.film_h, by_plugin.info.spp) == (ov["width"], ov["height"], ov["spp"])
    img_d, _ = O.render(by_defines.desc, pd, by_defines.border, rng=O.RNG_COUNTER)
    img_p, _ = O.render(by_plugin.desc, pp, by_plugin.border, rng=O.RNG_COUNTER)
    np.testing.assert_array_equal(img_p, img_d)


def test_override_checks_follow_monte_carlo_integrator():
    import mtsg
    with pytest.raises(RuntimeError, match="rrDepth"):
        mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {}, overrides=overrides_for(8, 8, 1, max_depth=3, rr_depth=0))
    with pytest.raises(RuntimeError, match="maxDepth"):
        mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {}, overrides=overrides_for(8, 8, 1, max_depth=0))
    with pytest.raises(RuntimeError, match="sampleCount"):
        mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {}, overrides=overrides_for(8, 8, 0))
