"""Environment emitter (src/emitters/envmap.cpp, mipmap.h) on the CPU side:
PFM / OpenEXR loading and the MIP pyramid, the sampling CDFs, and
sample-vs-pdf consistency of EnvironmentMap::sampleDirect.  The χ² check
mirrors the EmitterAdapter of the reference's
src/tests/test_chisquare.cpp:342-388,580-615 on the reference's own
data/tests/envmap.exr (PIZ-compressed HALF RGB, decoded by host/exr.cpp)
rotated 40 degrees about x, as data/tests/test_emitter.xml sets it up, and on
a seeded random map.  No reference test pins the decoded texel values (the
reference links OpenEXR): the decoder is checked by its own round trips
(NO / ZIP writers below) and by the image's structure."""
import ctypes as C
import math
import os

import numpy as np
import pytest

from conftest import REPO, SCENES
from test_bsdf_chisquare import PHI_BINS, THETA_BINS, chi2_pvalue, observed_counts

SIGNIFICANCE = 0.0025


def write_pfm(path, img):
    h, w, _ = img.shape
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode())
        f.write(np.ascontiguousarray(img[::-1]).astype("<f4").tobytes())


SCENE = """<scene version="0.5.0">
  <integrator type="path"/>
  <sensor type="perspective">
    <transform name="toWorld"><lookat origin="0, 0, 4" target="0, 0, 0" up="0, 1, 0"/></transform>
    <sampler type="independent"><integer name="sampleCount" value="4"/></sampler>
    <film type="hdrfilm"><integer name="width" value="32"/><integer name="height" value="24"/></film>
  </sensor>
  <emitter type="envmap">
    <string name="filename" value="{env}"/>
    <float name="scale" value="{scale}"/>
    <transform name="toWorld"><rotate x="1" angle="{angle}"/></transform>
  </emitter>
  <shape type="cube"><bsdf type="diffuse"/></shape>
</scene>
"""


def make_scene(tmp_path, img, scale=1.0, angle=40.0, env=None):
    import mtsg
    if env is None:
        env = tmp_path / "env.pfm"
        write_pfm(env, img)
    xml = tmp_path / "scene.xml"
    xml.write_text(SCENE.format(env=str(env), scale=scale, angle=angle))
    return mtsg.Scene(str(xml))


EXR = os.path.join(SCENES, "envmap.exr")   # the reference's data/tests/envmap.exr


def bind():
    from oracle import pyoracle as O
    L = O.lib()
    L.oracle_env_sample_direct_n.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.oracle_env_pdf_direct_n.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
    L.oracle_env_eval_n.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    return L, O._p


def env_pdf(scene, dirs):
    L, P = bind()
    dirs = np.ascontiguousarray(dirs, np.float32)
    out = np.zeros(len(dirs), np.float32)
    assert L.oracle_env_pdf_direct_n(scene.desc, len(dirs), P(dirs), P(out)) == 0
    return out


def env_eval(scene, dirs):
    L, P = bind()
    dirs = np.ascontiguousarray(dirs, np.float32)
    out = np.zeros((len(dirs), 3), np.float32)
    assert L.oracle_env_eval_n(scene.desc, len(dirs), P(dirs), None, None, P(out)) == 0
    return out


def test_pfm_orientation_and_bilinear_lookup(tmp_path):
    # a map whose top half is red, bottom half blue: +y must see red
    img = np.zeros((16, 32, 3), np.float32)
    img[:8, :, 0] = 2.0
    img[8:, :, 2] = 3.0
    sc = make_scene(tmp_path, img, scale=0.5, angle=0.0)
    v = env_eval(sc, np.array([[0, 1, 0], [0, -1, 0]], np.float32))
    np.testing.assert_allclose(v[0], [1.0, 0, 0], atol=1e-6)    # scale 0.5
    np.testing.assert_allclose(v[1], [0, 0, 1.5], atol=1e-6)


def test_half_precision_texels(tmp_path):
    # TMIPMap stores SpectrumHalf: 1/3 is returned rounded to binary16
    img = np.full((8, 16, 3), 1.0 / 3.0, np.float32)
    sc = make_scene(tmp_path, img, angle=0.0)
    v = env_eval(sc, np.array([[0.3, 0.5, -0.8]], np.float32))
    np.testing.assert_array_equal(v[0], np.float32(np.float16(1.0 / 3.0)))


def check_sampling_matches_pdf(sc, rng):
    L, P = bind()
    n = THETA_BINS * PHI_BINS * 1000
    u2 = rng.random((n, 2), dtype=np.float32)
    dirs = np.zeros((n, 3), np.float32); pdf = np.zeros(n, np.float32); val = np.zeros((n, 3), np.float32)
    ref = np.zeros(3, np.float32)   # inside the cube, inside the bounding sphere
    assert L.oracle_env_sample_direct_n(sc.desc, n, P(u2), P(ref), P(dirs), P(pdf), P(val)) == 0
    ok = pdf > 0
    assert ok.mean() > 0.999
    d = dirs[ok] / np.linalg.norm(dirs[ok], axis=1, keepdims=True)
    # sampled pdf == pdfDirect of the sampled direction, except where the tent
    # jitter pushes a sample across a pole (theta < 0 or > pi: the sampled
    # direction is mirrored and pdfDirect reads another row, as in Mitsuba)
    pd = env_pdf(sc, d[:20000])
    close = np.abs(pd - pdf[ok][:20000]) <= 2e-3 * np.abs(pdf[ok][:20000])
    a = math.radians(40.0)   # emitter-space y of the world direction (toWorld = rotate x 40)
    polar = np.abs(d[:20000, 1] * math.cos(a) + d[:20000, 2] * math.sin(a)) > 0.99
    assert np.all(close | polar)
    # expected counts: integral of pdfDirect over each (theta, phi) cell
    gl = 24
    x, w = np.polynomial.legendre.leggauss(gl)
    dth, dph = math.pi / THETA_BINS, 2 * math.pi / PHI_BINS
    ti = np.arange(THETA_BINS)[:, None, None, None]
    pj = np.arange(PHI_BINS)[None, :, None, None]
    th = (ti + 0.5 + 0.5 * x[None, None, :, None]) * dth
    ph = (pj + 0.5 + 0.5 * x[None, None, None, :]) * dph
    th, ph = np.broadcast_arrays(th, ph)
    q = np.stack([np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)], -1).reshape(-1, 3)
    p = env_pdf(sc, q).reshape(THETA_BINS, PHI_BINS, gl, gl).astype(np.float64)
    exp = (p * np.sin(th) * (w[:, None] * w[None, :]) * (0.25 * dth * dph)).sum((2, 3)) * n
    assert abs(exp.sum() / n - 1) < 0.02
    pval = chi2_pvalue(observed_counts(d), exp)
    assert pval >= SIGNIFICANCE, pval


def test_envmap_sampling_matches_pdf(tmp_path):
    rng = np.random.default_rng(11)
    base = rng.gamma(2.0, 1.0, size=(32, 64, 3)).astype(np.float32)
    # smooth it a little and add one bright region, like a sky with a sun
    base = 0.5 * base + 0.5 * np.roll(base, 1, axis=1)
    base[6:9, 40:44] *= 25.0
    check_sampling_matches_pdf(make_scene(tmp_path, base), rng)


def test_reference_envmap_sampling_matches_pdf(tmp_path):
    # the EmitterAdapter instance of test_chisquare.cpp:575-620 on
    # data/tests/test_emitter.xml's own map (envmap.exr, rotated 40 deg about x)
    check_sampling_matches_pdf(make_scene(tmp_path, None, env=EXR), np.random.default_rng(12))


def test_exr_decodes_the_reference_envmap():
    import mtsg
    img = mtsg.read_image(EXR)
    assert img.shape == (256, 512, 3)            # dataWindow (0,0)-(511,255), B/G/R HALF, PIZ
    assert np.isfinite(img).all() and img.min() > 0
    # HALF source: every value is exactly a binary16
    np.testing.assert_array_equal(img.astype(np.float16).astype(np.float32), img)
    # an image, not noise: neighbouring texels are ~10x closer in log
    # luminance than random pairs (a wrong Huffman / wavelet decode is noise)
    lum = np.log(img.mean(axis=2))
    d = np.abs(np.diff(lum, axis=1)).mean()
    rnd = np.abs(lum - np.random.default_rng(0).permutation(lum.ravel()).reshape(lum.shape)).mean()
    assert d < 0.15 * rnd
    # the ceiling (top rows) is brighter than the floor (bottom rows):
    # scanline order and the vertical orientation are right
    assert img[:32].mean() > img[-32:].mean()
    assert abs(float(img.mean()) - 0.3306) < 2e-3


def _write_exr(path, img, compression, half):
    """Minimal scanline OpenEXR writer (NO_COMPRESSION / ZIP), B/G/R."""
    import struct
    import zlib
    h, w, _ = img.shape
    def attr(name, typ, data):
        return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data
    ptype = 1 if half else 2
    chl = b"".join(c.encode() + b"\0" + struct.pack("<iB3xii", ptype, 0, 1, 1) for c in "BGR") + b"\0"
    hdr = (struct.pack("<II", 20000630, 2) + attr("channels", "chlist", chl) +
           attr("compression", "compression", bytes([compression])) +
           attr("dataWindow", "box2i", struct.pack("<4i", 0, 0, w - 1, h - 1)) +
           attr("displayWindow", "box2i", struct.pack("<4i", 0, 0, w - 1, h - 1)) +
           attr("lineOrder", "lineOrder", b"\0") + attr("pixelAspectRatio", "float", struct.pack("<f", 1)) +
           attr("screenWindowCenter", "v2f", struct.pack("<2f", 0, 0)) + attr("screenWindowWidth", "float", struct.pack("<f", 1)) + b"\0")
    lpc = 16 if compression == 3 else 1
    chunks = []
    dt = "<f2" if half else "<f4"
    for y0 in range(0, h, lpc):
        raw = b"".join(np.ascontiguousarray(img[y, :, c]).astype(dt).tobytes() for y in range(y0, min(h, y0 + lpc)) for c in (2, 1, 0))
        if compression == 3:
            b = np.frombuffer(raw, np.uint8)
            t = np.concatenate([b[0::2], b[1::2]])
            p = t.astype(np.int32)
            p[1:] = (t[1:].astype(np.int32) - t[:-1].astype(np.int32) + 128 + 256) & 255
            data = zlib.compress(p.astype(np.uint8).tobytes())
            if len(data) >= len(raw):   # the format stores a chunk raw when compression does not pay
                data = raw
        else:
            data = raw
        chunks.append(struct.pack("<ii", y0, len(data)) + data)
    off = len(hdr) + 8 * len(chunks)
    table = b""
    for c in chunks:
        table += struct.pack("<Q", off)
        off += len(c)
    open(path, "wb").write(hdr + table + b"".join(chunks))


@pytest.mark.parametrize("compression,half", [(0, True), (0, False), (3, True), (3, False)],
                         ids=["none-half", "none-float", "zip-half", "zip-float"])
def test_exr_round_trip(tmp_path, compression, half):
    import mtsg
    rng = np.random.default_rng(3)
    img = rng.gamma(2.0, 1.0, size=(37, 53, 3)).astype(np.float32)
    if half:
        img = img.astype(np.float16).astype(np.float32)
    p = tmp_path / "t.exr"
    _write_exr(str(p), img, compression, half)
    np.testing.assert_array_equal(mtsg.read_image(str(p)), img)


def test_env_glass_scene_loads():
    import mtsg
    sc = mtsg.Scene(os.path.join(SCENES, "env_glass.xml"), {"width": 32, "height": 18, "spp": 2})
    assert sc.info.n_emitters == 1 and sc.info.n_triangles > 100000
