"""GPU parity of `bitmap` textures against the oracle.

- Lookups through mtsg_tex_eval (BitmapTexture::eval, bitmap.cpp:431-499):
  the unfiltered level-0 lookups are bit-identical (no transcendentals; both
  sides without FMA contraction); the filtered ones (TMIPMap::eval,
  mipmap.h:633-722: trilinear and EWA with log2 / atan / sincos) agree to
  2e-4 relative (the bar of the environment-map lookups) for >= 99.9% of the
  lookups and to 5e-3 for all (EWA weight-LUT index steps, see the test).
- Renders of scenes/cbox_textured.xml (every filter and wrap mode, uv
  scale / offset, UV partials of camera hits, textured diffuse / plastic /
  roughplastic / twosided, a barycentric-uv mesh, the energy-conserving
  ScaleTexture) in counter mode: per-pixel L1 < 1e-3 of the mean.
- The same scene under the QMC samplers and with the two-level instancing
  build of the loader."""
import os

import numpy as np
import pytest

import mtsg
from oracle import pyoracle as O
from conftest import SCENES
from test_gpu_parity import check_render, render_pair

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tex_scene():
    s = mtsg.Scene(os.path.join(SCENES, "cbox_textured.xml"), {"width": 64, "height": 48, "spp": 8})
    g = mtsg.GPUScene(s, 0)
    yield s, g
    g.close()


def test_texture_lookups_match_oracle(tex_scene):
    s, g = tex_scene
    rng = np.random.default_rng(2024)
    n = 20000
    uv = rng.uniform(-1.5, 2.5, (n, 2)).astype(np.float32)
    # footprints from sub-texel to the whole texture, isotropic and skinny
    duv = (rng.normal(size=(n, 4)) * np.exp(rng.uniform(-9, 0.5, (n, 1)))).astype(np.float32)
    duv[: n // 4, 2:] = duv[: n // 4, :2] * np.float32(1e-3)   # strongly anisotropic
    for t in range(len(s.textures())):
        got, exp = g.tex_eval(t, uv), O.tex_eval(s.desc, t, uv)
        np.testing.assert_array_equal(got, exp)
        got, exp = g.tex_eval(t, uv, duv), O.tex_eval(s.desc, t, uv, duv)
        # an ulp of log2 / atan / sincos may move an ellipse's q across an
        # integer and pick the neighbouring entry of the 64-entry weight LUT
        # (a ~3% weight step on one texel): rare, bounded
        rel = np.abs(got - exp) / np.maximum(np.abs(exp), 1e-3)
        assert (rel < 2e-4).mean() >= 0.999, (rel >= 2e-4).mean()
        assert rel.max() < 5e-3, rel.max()


def test_textured_scene_parity(tex_scene):
    s, g = tex_scene
    _, c, gi = render_pair(s, g, max_depth=8)
    check_render(c, gi)


def test_textured_scene_depth_and_flags(tex_scene):
    s, g = tex_scene
    _, c, gi = render_pair(s, g, max_depth=2, hide_emitters=1)
    check_render(c, gi)
    _, c, gi = render_pair(s, g, max_depth=-1, strict_normals=1, seed=7)
    check_render(c, gi)


@pytest.mark.parametrize("sampler", ["ldsampler", "halton"])
def test_textured_scene_qmc_samplers(tmp_path, sampler):
    src = open(os.path.join(SCENES, "cbox_textured.xml")).read()
    src = src.replace('<sampler type="independent">', f'<sampler type="{sampler}">')
    p = tmp_path / "t.xml"
    p.write_text(src.replace('value="tex_', f'value="{SCENES}/tex_').replace('"bunny.ply"', f'"{SCENES}/bunny.ply"')
                 .replace('"envmap.exr"', f'"{SCENES}/envmap.exr"'))
    s = mtsg.Scene(str(p), {"width": 48, "height": 36, "spp": 8})
    g = mtsg.GPUScene(s, 0)
    _, c, gi = render_pair(s, g, max_depth=6)
    check_render(c, gi)
    g.close()


def test_textured_instances_parity(tmp_path):
    """Textured shapes inside a shapegroup: uv and both tangents mapped by each
    instance's toWorld (instance.cpp:146-160), filtered at camera hits."""
    xml = f"""<scene version="0.5.0">
  <integrator type="path"><integer name="maxDepth" value="6"/></integrator>
  <sensor type="perspective"><float name="fov" value="40"/>
    <transform name="toWorld"><lookat origin="0, 1.2, 4" target="0, 0, 0" up="0, 1, 0"/></transform>
    <sampler type="independent"><integer name="sampleCount" value="8"/></sampler>
    <film type="hdrfilm"><integer name="width" value="48"/><integer name="height" value="36"/></film></sensor>
  <texture type="bitmap" id="chk"><string name="filename" value="{SCENES}/tex_checker.png"/>
    <float name="uscale" value="2"/></texture>
  <shape type="shapegroup" id="g">
    <shape type="cube"><bsdf type="diffuse"><ref name="reflectance" id="chk"/></bsdf></shape>
  </shape>
  <shape type="instance"><ref id="g"/><transform name="toWorld"><scale value="0.4"/><rotate y="1" angle="30"/>
    <translate x="-0.6"/></transform></shape>
  <shape type="instance"><ref id="g"/><transform name="toWorld"><scale x="0.3" y="0.5" z="0.3"/><rotate x="1" angle="20"/>
    <translate x="0.6"/></transform></shape>
  <shape type="rectangle"><transform name="toWorld"><scale value="3"/><rotate x="1" angle="-90"/><translate y="-0.6"/>
    </transform><bsdf type="diffuse"><ref name="reflectance" id="chk"/></bsdf></shape>
  <shape type="rectangle"><transform name="toWorld"><rotate x="1" angle="90"/><translate y="2.5"/></transform>
    <emitter type="area"><rgb name="radiance" value="4, 4, 4"/></emitter></shape>
</scene>"""
    p = tmp_path / "inst.xml"
    p.write_text(xml)
    for inst in ("flatten", "two-level"):
        s = mtsg.Scene(str(p), instancing=inst)
        g = mtsg.GPUScene(s, 0)
        _, c, gi = render_pair(s, g)
        check_render(c, gi)
        g.close()
