"""hdrfilm crop windows (src/librender/film.cpp:36-48, src/films/hdrfilm.cpp:57,352):
the render covers the crop rectangle of a film whose projection stays the
full film's, so a cropped scene renders what the full scene renders on that
rectangle (params tile_x/y/w/h), bit for bit with the oracle's fixed splat
order.  The plugin route passes the crop Mitsuba holds in memory
(MTSH_OVERRIDE_FILM_CROP), and invalid windows fail with film.cpp's message."""
import os

import numpy as np
import pytest

from conftest import SCENES

CROP = dict(x=24, y=16, w=40, h=24)


def cropped_xml(tmp_path, src="cbox.xml", crop=CROP):
    s = open(os.path.join(SCENES, src)).read()
    film = '<film type="hdrfilm">'
    assert film in s
    s = s.replace(film, film + f'<integer name="cropOffsetX" value="{crop["x"]}"/><integer name="cropOffsetY" '
                  f'value="{crop["y"]}"/><integer name="cropWidth" value="{crop["w"]}"/><integer name="cropHeight" '
                  f'value="{crop["h"]}"/>', 1)
    s = s.replace('value="bunny.ply"', f'value="{os.path.join(SCENES, "bunny.ply")}"')
    p = tmp_path / ("crop_" + src)
    p.write_text(s)
    return str(p)


DEFS = {"width": 96, "height": 64, "spp": 3, "maxDepth": 5}


def test_crop_window_renders_the_rectangle_of_the_full_film(tmp_path):
    import mtsg
    from oracle import pyoracle as O
    cropped = mtsg.Scene(cropped_xml(tmp_path), DEFS)
    full = mtsg.Scene(os.path.join(SCENES, "cbox.xml"), DEFS)
    pc = cropped.params()
    assert (pc.tile_x, pc.tile_y, pc.tile_w, pc.tile_h) == (CROP["x"], CROP["y"], CROP["w"], CROP["h"])
    assert (cropped.info.film_w, cropped.info.film_h) == (96, 64)
    pf = full.params(tile_x=CROP["x"], tile_y=CROP["y"], tile_w=CROP["w"], tile_h=CROP["h"])
    img_c, st = O.render(cropped.desc, pc, cropped.border, rng=O.RNG_COUNTER)
    img_f, _ = O.render(full.desc, pf, full.border, rng=O.RNG_COUNTER)
    assert img_c.shape == (CROP["h"] + 2 * cropped.border, CROP["w"] + 2 * cropped.border, 5)
    assert st.samples == CROP["w"] * CROP["h"] * 3
    assert img_c[..., 4].sum() > 0
    np.testing.assert_array_equal(img_c, img_f)


def test_plugin_crop_override_equals_the_xml_crop(tmp_path):
    import mtsg
    from oracle import pyoracle as O
    from test_plugin_overrides import overrides_for
    by_xml = mtsg.Scene(cropped_xml(tmp_path), DEFS)
    ov = overrides_for(96, 64, 3, max_depth=5)
    ov.mask |= mtsg.MTSH_OVERRIDE_FILM_CROP
    ov.crop_x, ov.crop_y, ov.crop_width, ov.crop_height = CROP["x"], CROP["y"], CROP["w"], CROP["h"]
    by_plugin = mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {}, overrides=ov)
    a, b = by_xml.params(), by_plugin.params()
    for f in ("tile_x", "tile_y", "tile_w", "tile_h", "spp", "max_depth"):
        assert getattr(a, f) == getattr(b, f), f
    img_x, _ = O.render(by_xml.desc, a, by_xml.border, rng=O.RNG_COUNTER)
    img_p, _ = O.render(by_plugin.desc, b, by_plugin.border, rng=O.RNG_COUNTER)
    np.testing.assert_array_equal(img_x, img_p)


def test_film_size_override_keeps_or_refuses_the_xml_crop(tmp_path):
    import mtsg
    from test_plugin_overrides import overrides_for
    # the same size: the XML's crop stays
    xml = cropped_xml(tmp_path)
    s = mtsg.Scene(xml, {"width": 96, "height": 64}, overrides=overrides_for(96, 64, 2))
    p = s.params()
    assert (p.tile_x, p.tile_y, p.tile_w, p.tile_h) == (CROP["x"], CROP["y"], CROP["w"], CROP["h"])
    # another size without the crop: refused (the crop would not fit)
    with pytest.raises(RuntimeError, match="crop"):
        mtsg.Scene(xml, {"width": 96, "height": 64}, overrides=overrides_for(48, 32, 2))


@pytest.mark.parametrize("crop", [dict(x=-1, y=0, w=8, h=8), dict(x=0, y=0, w=0, h=8),
                                  dict(x=90, y=0, w=8, h=8), dict(x=0, y=60, w=8, h=8)])
def test_invalid_crop_windows_fail_like_film_cpp(tmp_path, crop):
    import mtsg
    with pytest.raises(RuntimeError, match="Invalid crop window specification"):
        mtsg.Scene(cropped_xml(tmp_path, crop=crop), DEFS)
