"""`bitmap` textures on the host and in the oracle.

- The PNG reader (Bitmap::readPNG, src/libcore/bitmap.cpp:2460-2560) against
  the arrays tools/gen_textures.py encodes: 8/16-bit, gray / RGB / RGBA /
  4-bit palette, every scanline filter type, and the gamma the reference
  assigns (sRGB chunk, gAMA chunk, sRGB by default), converted as
  FormatConverter does (fmtconv.cpp:1093-1160).
- The MIP pyramid (TMIPMap constructor, mipmap.h:155-302) against an
  independent numpy restatement of the 2-lobe Lanczos resampler
  (rfilter.h:107-460) for every boundary condition, with the [0, maxValue]
  clamp and the half-precision storage.
- The oracle's level-0 lookups (evalTexel / evalBox / evalBilinear,
  mipmap.h:503-596) against numpy over every wrap mode.
- The scene loader: texture parameters, ensureEnergyConservation's
  ScaleTexture (bsdf.cpp:88-113), plastic's sampling weight from the texture
  average (plastic.cpp:199-201), error messages.
- An oracle render of a constant texture equals the constant reflectance.

No reference-held fixture covers textures (data/tests has no textured scene),
so the loader and lookup values are pinned by these restatements only."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import mtsg
from oracle import pyoracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(REPO, "scenes")
sys.path.insert(0, os.path.join(REPO, "tools"))
import gen_textures as G  # noqa: E402


def srgb_to_linear(v):
    v = v.astype(np.float32)
    lo = v * np.float32(1.0 / 12.92)
    hi = np.power((v + np.float32(0.055)) * np.float32(1.0 / 1.055), np.float32(2.4)).astype(np.float32)
    return np.where(v <= np.float32(0.04045), lo, hi)


def test_png_decodes_every_format(tmp_path):
    G.main(str(tmp_path))
    inv255 = np.float32(1.0) / np.float32(255.0)
    a = mtsg.texture_image(str(tmp_path / "tex_checker.png"), 1.0)
    np.testing.assert_array_equal(a, G.checker().astype(np.float32) * inv255)
    a = mtsg.texture_image(str(tmp_path / "tex_rgba.png"), 1.0)   # alpha dropped (ERGBA -> ERGB)
    np.testing.assert_array_equal(a, G.rgba()[..., :3].astype(np.float32) * inv255)
    a = mtsg.texture_image(str(tmp_path / "tex_gray16.png"), 1.0)  # luminance broadcast
    g = G.gray16()[..., 0].astype(np.float32) * (np.float32(1.0) / np.float32(65535.0))
    np.testing.assert_array_equal(a, np.repeat(g[..., None], 3, -1))
    idx, pal = G.palette4()
    a = mtsg.texture_image(str(tmp_path / "tex_palette.png"), 1.0)
    np.testing.assert_array_equal(a, pal[idx[..., 0]].astype(np.float32) * inv255)


def test_png_gamma_as_the_reference_assigns_it(tmp_path):
    G.main(str(tmp_path))
    inv255 = np.float32(1.0) / np.float32(255.0)
    # no colour chunk and the sRGB chunk: sRGB (bitmap.cpp:2534-2541)
    for name, src in (("tex_checker.png", G.checker()), ("tex_rgba.png", G.rgba()[..., :3])):
        a = mtsg.texture_image(str(tmp_path / name))
        np.testing.assert_allclose(a, srgb_to_linear(src.astype(np.float32) * inv255), rtol=2e-7, atol=1e-9)
    # gAMA 0.45455 -> m_gamma = 1 / 0.45455, undoGamma = pow(v, gamma)
    a = mtsg.texture_image(str(tmp_path / "tex_gray16.png"))
    g = G.gray16()[..., 0].astype(np.float32) * (np.float32(1.0) / np.float32(65535.0))
    gamma = np.float32(1.0) / np.float32(0.45455)
    np.testing.assert_allclose(a[..., 0], np.power(g, gamma), rtol=2e-6)
    # the texture's `gamma` parameter overrides the file (Bitmap::setGamma)
    a = mtsg.texture_image(str(tmp_path / "tex_checker.png"), 2.0)
    np.testing.assert_allclose(a, np.power(G.checker().astype(np.float32) * inv255, 2.0), rtol=2e-7)


def test_png_rejects_interlaced_and_corrupt_files(tmp_path):
    G.write_png(str(tmp_path / "ok.png"), G.checker(8, 8), 2, 8)
    data = bytearray(open(tmp_path / "ok.png", "rb").read())
    bad = bytearray(data)
    bad[28] = 1   # IHDR interlace method
    open(tmp_path / "il.png", "wb").write(bad)
    with pytest.raises(RuntimeError, match="interlaced"):
        mtsg.texture_image(str(tmp_path / "il.png"))
    open(tmp_path / "trunc.png", "wb").write(data[:60])
    with pytest.raises(RuntimeError):
        mtsg.texture_image(str(tmp_path / "trunc.png"))


# ---------------------------------------------------------------------------
# MIP pyramid vs an independent restatement of the Lanczos resampler
# ---------------------------------------------------------------------------
def lanczos2(x):
    x = np.abs(x)
    x1 = np.pi * x
    x2 = x1 / 2
    with np.errstate(invalid="ignore", divide="ignore"):
        v = np.sin(x1) * np.sin(x2) / (x1 * x2)
    return np.where(x < 1e-4, 1.0, np.where(x > 2, 0.0, v))


def resample_axis(a, n_out, bc, vmax):
    """Resample axis 0 of a (n_in, ...) array (Resampler in resampling mode)."""
    n_in = a.shape[0]
    scale = n_in / n_out if n_out < n_in else 1.0
    radius = 2.0 * scale
    taps = int(np.ceil(radius * 2))
    out = np.zeros((n_out,) + a.shape[1:])
    for i in range(n_out):
        center = (i + 0.5) / n_out * n_in
        start = int(np.floor(center - radius + 0.5))
        pos = start + np.arange(taps)
        w = lanczos2((pos + 0.5 - center) / scale)
        w = w / w.sum()
        vals = []
        for p in pos:
            if 0 <= p < n_in:
                vals.append(a[p])
            elif bc == mtsg.WRAP_CLAMP:
                vals.append(a[min(max(p, 0), n_in - 1)])
            elif bc == mtsg.WRAP_REPEAT:
                vals.append(a[p % n_in])
            elif bc == mtsg.WRAP_MIRROR:
                q = p % (2 * n_in)
                vals.append(a[2 * n_in - q - 1 if q >= n_in else q])
            else:
                vals.append(np.full(a.shape[1:], 0.0 if bc == mtsg.WRAP_ZERO else 1.0))
        out[i] = np.clip(np.tensordot(w, np.array(vals), 1), 0, vmax)
    return out


@pytest.mark.parametrize("bc", [mtsg.WRAP_CLAMP, mtsg.WRAP_REPEAT, mtsg.WRAP_MIRROR, mtsg.WRAP_ZERO, mtsg.WRAP_ONE])
def test_mipmap_levels_match_lanczos_restatement(bc):
    rng = np.random.default_rng(7 + bc)
    img = rng.uniform(-0.2, 1.6, (7, 13, 3)).astype(np.float32)
    levels, hdr, avg, mx = mtsg.build_mipmap(img, mtsg.MIP_EWA, bc, mtsg.WRAP_CLAMP if bc != 1 else mtsg.WRAP_MIRROR, 1.0, 20.0)
    assert hdr.levels == 5 and [hdr.level_w[l] for l in range(5)] == [13, 7, 4, 2, 1]
    assert [hdr.level_h[l] for l in range(5)] == [7, 4, 2, 1, 1]
    lvl0 = np.maximum(img, 0)   # negative values clamped, level 0 not clamped to maxValue
    np.testing.assert_array_equal(levels[0], lvl0.astype(np.float16).astype(np.float32))
    np.testing.assert_allclose(avg, lvl0.reshape(-1, 3).mean(0), rtol=1e-6)
    np.testing.assert_array_equal(mx, lvl0.reshape(-1, 3).max(0))
    bcv = mtsg.WRAP_CLAMP if bc != 1 else mtsg.WRAP_MIRROR
    cur = lvl0.astype(np.float64)
    for l in range(1, 5):
        h, w = cur.shape[:2]
        nw, nh = max(1, (w + 1) // 2), max(1, (h + 1) // 2)
        if nw != w:
            cur = resample_axis(cur.transpose(1, 0, 2), nw, bc, 1.0).transpose(1, 0, 2)
        if nh != h:
            cur = resample_axis(cur, nh, bcv, 1.0)
        # half storage: within one half ulp of the float result
        np.testing.assert_allclose(levels[l], cur, rtol=1.2e-3, atol=1e-6)
        assert levels[l].max() <= 1.0 and levels[l].min() >= 0.0


def test_bilinear_and_nearest_pyramids_keep_level_zero():
    img = np.random.default_rng(3).uniform(0, 1, (9, 5, 3)).astype(np.float32)
    for f in (mtsg.MIP_NEAREST, mtsg.MIP_BILINEAR):
        levels, hdr, _, _ = mtsg.build_mipmap(img, f)
        assert hdr.levels == 1 and hdr.max_anisotropy == 1.0
    _, hdr, _, _ = mtsg.build_mipmap(img, mtsg.MIP_TRILINEAR, max_anisotropy=20.0)
    assert hdr.levels == 5 and hdr.max_anisotropy == 1.0   # only EWA keeps maxAnisotropy (bitmap.cpp:234-235)


# ---------------------------------------------------------------------------
# Scene loading and the oracle's lookups
# ---------------------------------------------------------------------------
def _scene(tmp_path, bsdf_xml, extra="", w=16, h=12, spp=2):
    G.main(str(tmp_path))
    xml = f"""<scene version="0.5.0">
  <integrator type="path"><integer name="maxDepth" value="4"/></integrator>
  <sensor type="perspective"><float name="fov" value="45"/>
    <transform name="toWorld"><lookat origin="0, 0, 3" target="0, 0, 0" up="0, 1, 0"/></transform>
    <sampler type="independent"><integer name="sampleCount" value="{spp}"/></sampler>
    <film type="hdrfilm"><integer name="width" value="{w}"/><integer name="height" value="{h}"/>
      <rfilter type="box"/></film></sensor>
  {extra}
  <shape type="rectangle">{bsdf_xml}</shape>
  <shape type="rectangle"><transform name="toWorld"><rotate x="1" angle="180"/><translate z="4"/></transform>
    <emitter type="area"><rgb name="radiance" value="3, 3, 3"/></emitter></shape>
</scene>"""
    p = tmp_path / "s.xml"
    p.write_text(xml)
    return mtsg.Scene(str(p))


def _bsdfs(scene):
    from test_scene_kdtree import _bsdfs as b
    return b(scene)


def level0_lookup(img, u, v, wu, wv, nearest):
    """evalBox(0) / evalBilinear(0) in float64 with the wrap modes."""
    h, w = img.shape[:2]

    def texel(x, y):
        out = np.zeros(x.shape + (3,))
        ok = np.ones(x.shape, bool)
        const = np.zeros(x.shape)
        for coord, n, mode, ax in ((x, w, wu, 0), (y, h, wv, 1)):
            c = coord.copy()
            out_of = (c < 0) | (c >= n)
            if mode == mtsg.WRAP_REPEAT:
                c = c % n
            elif mode == mtsg.WRAP_CLAMP:
                c = np.clip(c, 0, n - 1)
            elif mode == mtsg.WRAP_MIRROR:
                c = c % (2 * n)
                c = np.where(c >= n, 2 * n - c - 1, c)
            else:
                newly = out_of & ok
                const = np.where(newly, 0.0 if mode == mtsg.WRAP_ZERO else 1.0, const)
                ok &= ~out_of
                c = np.clip(c, 0, n - 1)
            if ax == 0:
                x = c
            else:
                y = c
        vals = img[y, x]
        return np.where(ok[..., None], vals, const[..., None])

    f = np.float32
    if nearest:
        return texel(np.floor(u.astype(f) * f(w)).astype(int), np.floor(v.astype(f) * f(h)).astype(int))
    # texel-space coordinates in single precision, as the reference computes them
    uu = (u.astype(f) * f(w) - f(0.5)).astype(np.float64)
    vv = (v.astype(f) * f(h) - f(0.5)).astype(np.float64)
    x0, y0 = np.floor(uu).astype(int), np.floor(vv).astype(int)
    dx, dy = (uu - x0)[..., None], (vv - y0)[..., None]
    return (texel(x0, y0) * (1 - dx) * (1 - dy) + texel(x0, y0 + 1) * (1 - dx) * dy +
            texel(x0 + 1, y0) * dx * (1 - dy) + texel(x0 + 1, y0 + 1) * dx * dy)


@pytest.mark.parametrize("wrap", ["repeat", "clamp", "mirror", "zero", "one"])
@pytest.mark.parametrize("filt", ["nearest", "bilinear"])
def test_oracle_level0_lookups(tmp_path, wrap, filt):
    sc = _scene(tmp_path, f"""<bsdf type="diffuse"><texture type="bitmap" name="reflectance">
        <string name="filename" value="tex_checker.png"/><string name="filterType" value="{filt}"/>
        <string name="wrapMode" value="{wrap}"/></texture></bsdf>""")
    (t,) = sc.textures()
    img = G.checker().astype(np.float32) * (np.float32(1) / np.float32(255))
    img = srgb_to_linear(img).astype(np.float16).astype(np.float64)
    rng = np.random.default_rng(11)
    uv = rng.uniform(-1.7, 2.6, (4000, 2)).astype(np.float32)
    got = O.tex_eval(sc.desc, 0, uv)
    codes = {"repeat": 1, "clamp": 0, "mirror": 2, "zero": 3, "one": 4}
    exp = level0_lookup(img, uv[:, 0].astype(np.float64), uv[:, 1].astype(np.float64), codes[wrap], codes[wrap], filt == "nearest")
    np.testing.assert_allclose(got, exp, rtol=2e-6, atol=2e-6)
    # filtered lookups of nearest / bilinear textures are the same level-0 lookups
    duv = rng.uniform(-0.2, 0.2, (4000, 4)).astype(np.float32)
    np.testing.assert_array_equal(O.tex_eval(sc.desc, 0, uv, duv), got)


def test_trilinear_and_ewa_blend_levels(tmp_path):
    sc = _scene(tmp_path, """<bsdf type="diffuse"><texture type="bitmap" name="reflectance">
        <string name="filename" value="tex_checker.png"/></texture></bsdf>""")
    uv = np.full((5, 2), 0.37, np.float32)
    tiny = np.zeros((5, 4), np.float32)
    tiny[:, 0] = tiny[:, 3] = 1e-5
    # footprints far below a texel: bilinear level 0
    np.testing.assert_array_equal(O.tex_eval(sc.desc, 0, uv, tiny), O.tex_eval(sc.desc, 0, uv))
    # a footprint covering the whole texture: the average of the image
    huge = np.zeros((5, 4), np.float32)
    huge[:, 0] = huge[:, 3] = 4.0
    v = O.tex_eval(sc.desc, 0, uv, huge)
    (t,) = sc.textures()
    assert np.abs(v[0] - np.array(t.average)).max() < 0.05
    # anisotropic footprints stay finite and within [0, maxValue] (Lanczos
    # ringing may lift resampled levels above the level-0 maximum)
    rng = np.random.default_rng(5)
    duv = (rng.normal(size=(3000, 4)) * np.exp(rng.uniform(-8, 0, (3000, 1)))).astype(np.float32)
    v = O.tex_eval(sc.desc, 0, rng.uniform(0, 1, (3000, 2)).astype(np.float32), duv)
    assert np.isfinite(v).all() and v.min() >= 0 and v.max() <= 1.0


def test_loader_texture_parameters_and_energy_conservation(tmp_path):
    sc = _scene(tmp_path, """<bsdf type="plastic"><texture type="bitmap" name="diffuseReflectance">
        <string name="filename" value="tex_rgba.png"/><string name="wrapModeU" value="mirror"/>
        <string name="wrapModeV" value="one"/><float name="uvscale" value="2"/><float name="voffset" value="0.25"/>
        <float name="uscale" value="3"/></texture></bsdf>""",
                extra="""<texture type="bitmap" id="hdr"><string name="filename" value="%s"/></texture>
        <bsdf type="diffuse" id="d"><ref name="reflectance" id="hdr"/></bsdf>""" % os.path.join(SCENES, "envmap.exr"))
    tex = sc.textures()
    b = _bsdfs(sc)
    hdr = [t for t in tex if max(t.maximum) > 1]
    assert len(hdr) == 2   # the shared texture and the BSDF's scaled copy
    scaled = [t for t in hdr if t.scale != 1.0]
    assert len(scaled) == 1
    assert abs(scaled[0].scale - 0.99 / max(scaled[0].maximum)) < 1e-6 * scaled[0].scale
    d = [x for x in b if x.type == 1 and x.texture]
    assert tex[d[0].texture - 1].scale == scaled[0].scale
    p = [x for x in b if x.type == 5][0]
    t = tex[p.texture - 1]
    assert (t.mip.wrap_u, t.mip.wrap_v, t.mip.filter) == (mtsg.WRAP_MIRROR, mtsg.WRAP_ONE, mtsg.MIP_EWA)
    assert tuple(t.uv_scale) == (3.0, 2.0) and tuple(t.uv_offset) == (0.0, 0.25)
    assert abs(t.mip.max_anisotropy - 20.0) < 1e-6
    lum = lambda v: v[0] * 0.212671 + v[1] * 0.715160 + v[2] * 0.072169
    assert abs(p.spec_sampling_weight - 1.0 / (lum(t.average) + 1.0)) < 1e-6   # sAvg = 1


@pytest.mark.parametrize("bsdf,msg", [
    ("""<bsdf type="roughconductor"><texture type="bitmap" name="specularReflectance">
        <string name="filename" value="tex_checker.png"/></texture></bsdf>""", "outside this build's scope"),
    ("""<bsdf type="diffuse"><texture type="bitmap" name="reflectance"><string name="filename" value="tex_checker.png"/>
        <string name="filterType" value="box"/></texture></bsdf>""", "Unknown filter type 'box'"),
    ("""<bsdf type="diffuse"><texture type="bitmap" name="reflectance"><string name="filename" value="tex_checker.png"/>
        <string name="wrapMode" value="wrap"/></texture></bsdf>""", "Unknown wrap mode 'wrap'"),
    ("""<bsdf type="diffuse"><texture type="checkerboard" name="reflectance"/></bsdf>""", "outside this build's scope"),
    ("""<bsdf type="diffuse"><texture type="bitmap" name="reflectance"><string name="filename" value="tex_checker.png"/>
        <string name="channel" value="r"/></texture></bsdf>""", "channel"),
])
def test_loader_rejects_what_the_device_does_not_evaluate(tmp_path, bsdf, msg):
    with pytest.raises(RuntimeError, match=msg):
        _scene(tmp_path, bsdf)


def test_constant_texture_renders_like_the_constant(tmp_path):
    """A 2x2 texture of one half-exact value renders as that constant reflectance
    (bilinear weights sum to one up to rounding)."""
    G.write_png(str(tmp_path / "const.png"), np.full((2, 2, 3), 128, np.uint8), 2, 8)
    val = float(srgb_to_linear(np.float32(128) * (np.float32(1) / np.float32(255))).astype(np.float16))
    a = _scene(tmp_path, f"""<bsdf type="diffuse"><texture type="bitmap" name="reflectance">
        <string name="filename" value="{tmp_path / 'const.png'}"/></texture></bsdf>""", w=24, h=18, spp=4)
    b = _scene(tmp_path, f"""<bsdf type="diffuse"><rgb name="reflectance" value="{val}"/></bsdf>""", w=24, h=18, spp=4)
    ia, _ = O.render(a.desc, a.params(), a.border, rng=O.RNG_COUNTER)
    ib, _ = O.render(b.desc, b.params(), b.border, rng=O.RNG_COUNTER)
    ra, rb = mtsg.develop(ia), mtsg.develop(ib)
    assert rb.mean() > 0
    assert np.abs(ra - rb).max() < 1e-5 * max(1.0, rb.max())


def test_textured_cbox_loads_and_renders():
    sc = mtsg.Scene(os.path.join(SCENES, "cbox_textured.xml"), {"width": 24, "height": 18, "spp": 2})
    tex = sc.textures()
    assert len(tex) == 6   # checker, rgba, palette, gray16, envmap + its energy-conserving copy
    assert sorted(t.mip.filter for t in tex).count(mtsg.MIP_EWA) == 3
    img, _ = O.render(sc.desc, sc.params(), sc.border, rng=O.RNG_COUNTER)
    rgb = mtsg.develop(img)
    assert np.isfinite(rgb).all() and rgb.mean() > 0.01


def test_png_decoder_agrees_with_pil(tmp_path):
    """An independent decoder: PIL (libpng-compatible, importable here) reads
    the committed PNG fixtures and PNGs that PIL itself encodes (with its own
    filter choices and zlib streams) -- the host reader must give the same
    8/16-bit values (raw, gamma 1) as PIL for every one of them."""
    from PIL import Image
    inv255 = np.float32(1.0) / np.float32(255.0)
    files = [os.path.join(SCENES, f) for f in ("tex_checker.png", "tex_rgba.png", "tex_palette.png", "tex_gray16.png")]
    rng = np.random.default_rng(9)
    for mode, arr in (("RGB", rng.integers(0, 256, (29, 41, 3), dtype=np.uint8)),
                      ("RGBA", rng.integers(0, 256, (17, 23, 4), dtype=np.uint8)),
                      ("L", rng.integers(0, 256, (31, 19), dtype=np.uint8))):
        p = tmp_path / f"pil_{mode}.png"
        Image.fromarray(arr, mode).save(p, optimize=True)
        files.append(str(p))
    p = tmp_path / "pil_P.png"
    Image.fromarray(rng.integers(0, 256, (21, 27, 3), dtype=np.uint8), "RGB").convert("P", palette=Image.ADAPTIVE,
                                                                                     colors=16).save(p, bits=4)
    files.append(str(p))
    p = tmp_path / "pil_I16.png"
    Image.fromarray(rng.integers(0, 65536, (13, 11), dtype=np.uint16)).save(p)
    files.append(str(p))
    for f in files:
        im = Image.open(f)
        got = mtsg.texture_image(f, 1.0)
        if im.mode in ("I;16", "I;16B", "I"):
            g = np.asarray(im).astype(np.float32) * (np.float32(1.0) / np.float32(65535.0))
            want = np.repeat(g[..., None], 3, -1)
        else:
            a = np.asarray(im.convert("RGBA" if "A" in im.mode or im.mode == "P" else "RGB"))[..., :3]
            if im.mode == "L":
                a = np.repeat(np.asarray(im)[..., None], 3, -1)
            want = a.astype(np.float32) * inv255
        np.testing.assert_array_equal(got, want, err_msg=f)
