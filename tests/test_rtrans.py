"""roughplastic's rough dielectric transmittance (src/bsdfs/rtrans.h).

The reference ships RoughTransmittance as precomputed tables
(data/microfacet/*.dat) validated against quadrature by
src/tests/test_rtrans.cpp (|table - integral| <= 1e-3).  This build computes
the material's slice by quadrature instead (my-mitsuba_amd/host/rtrans.cpp).
Parity is pinned against a subset of the reference's table nodes, kept as data
in tests/golden/rtrans_nodes.json (tools/extract_rtrans_nodes.py):

- external block (eta > 1; the per-hit T12/T21 and the sampling split): every
  theta sample of every kept node within 1.5e-3, diffuse within 1e-3;
- internal block (eta < 1; enters roughplastic only through the scalar Fdr):
  the reference's adaptive integrator left some thin transmissive regions at
  0 (e.g. GGX, eta 1/1.4216, alpha 0.1625, cos 0.236: table 0.0, converged
  quadrature 0.0253), so its diffuse transmittance is matched within 1.2e-2
  (parity partial there; the quadrature is the converged value).
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

import mtsg
from conftest import GOLDEN, SCENES

N = 100


def _lib():
    L = mtsg.host_lib()
    L.mtsh_rough_transmittance.argtypes = [C.c_int, C.c_float, C.c_float, C.c_int, C.c_void_p, C.c_void_p]
    return L


def slice_(dist, alpha, eta):
    tr = (C.c_float * N)()
    df = C.c_float()
    assert _lib().mtsh_rough_transmittance(dist, C.c_float(alpha), C.c_float(eta), N, tr, C.byref(df)) == 0
    return np.array(tr[:], np.float64), df.value


GOLD = json.load(open(os.path.join(GOLDEN, "rtrans_nodes.json")))


@pytest.mark.parametrize("name", ["beckmann", "ggx", "phong"])
def test_external_block_matches_reference_tables(name):
    t = GOLD["tables"][name]
    assert t["theta_samples"] == N
    for node in t["nodes"]:
        if node["eta"] < 1:
            continue
        tr, df = slice_(t["distribution"], node["alpha"], node["eta"])
        err = np.abs(tr - np.array(node["trans"])).max()
        assert err <= 1.5e-3, (name, node["eta"], node["alpha"], err)
        assert abs(df - node["diffuse"]) <= 1e-3, (name, node["eta"], node["alpha"], df, node["diffuse"])


@pytest.mark.parametrize("name", ["beckmann", "ggx", "phong"])
def test_internal_block_diffuse(name):
    t = GOLD["tables"][name]
    for node in t["nodes"]:
        if node["eta"] >= 1:
            continue
        _, df = slice_(t["distribution"], node["alpha"], node["eta"])
        assert abs(df - node["diffuse"]) <= 1.2e-2, (name, node["eta"], node["alpha"], df, node["diffuse"])


def test_invalid_arguments():
    tr = (C.c_float * N)()
    L = _lib()
    assert L.mtsh_rough_transmittance(7, C.c_float(0.1), C.c_float(1.5), N, tr, None) != 0
    assert L.mtsh_rough_transmittance(0, C.c_float(0.0), C.c_float(1.5), N, tr, None) != 0
    assert L.mtsh_rough_transmittance(0, C.c_float(0.1), C.c_float(1.5), 1, tr, None) != 0


def test_smooth_limit_is_fresnel():
    # alpha -> 0: T(mu) -> 1 - F(mu) and the diffuse transmittance -> 1 - Fdr
    eta = 1.5
    tr, df = slice_(0, 1e-4, eta)
    mu = (np.arange(N) / (N - 1)) ** 4

    def F(c):
        s = np.sqrt(np.maximum(0, 1 - (1 - c * c) / eta ** 2))
        rs = (c - eta * s) / (c + eta * s)
        rp = (eta * c - s) / (eta * c + s)
        return 0.5 * (rs * rs + rp * rp)
    sel = mu > 0.05
    np.testing.assert_allclose(tr[sel], 1 - F(mu[sel]), atol=2e-3)
    x = (np.arange(200000) + 0.5) / 200000
    assert abs(df - (1 - (2 * x * F(x)).mean())) < 1e-3


def _bsdfs(scene):
    from test_scene_kdtree import _bsdfs as b
    return b(scene)


def test_roughplastic_records():
    s = mtsg.Scene(os.path.join(SCENES, "cbox_roughplastic.xml"), {"width": 16, "height": 16, "spp": 1})
    rp = [b for b in _bsdfs(s) if b.type == 7]
    assert len(rp) == 6   # 5 materials + the twosided front record (a copy of its nested BRDF)
    for b in rp:
        assert b.smooth == 1 and b.ref_n_zero == b.twosided and b.alpha_u == b.alpha_v   # twosided: EBackSide
        tr = np.array(b.rtrans[:])
        assert 0 < b.fdr_int < 1 and (tr >= 0).all() and (tr <= 1).all() and tr[-1] > 0.8
        exp, df_int = slice_(b.distribution, b.alpha_u, b.ior_eta)[0], slice_(b.distribution, b.alpha_u, b.ior_inv_eta)[1]
        np.testing.assert_array_equal(tr, exp.astype(np.float32))
        assert abs(b.fdr_int - (1 - df_int)) < 1e-6


def _load(tmp_path, bsdf):
    p = tmp_path / "s.xml"
    p.write_text(open(os.path.join(SCENES, "cbox.xml")).read().replace(
        '<bsdf type="diffuse" id="white">', bsdf + '\n<bsdf type="diffuse" id="white">', 1))
    return mtsg.Scene(str(p), {"width": 8, "height": 8, "spp": 1})


@pytest.mark.parametrize("bsdf,msg", [
    ('<bsdf type="roughplastic" id="x"><float name="alphaU" value="0.1"/><float name="alphaV" value="0.3"/></bsdf>',
     "anisotropic"),
    ('<bsdf type="roughplastic" id="x"><string name="distribution" value="phong"/><float name="alpha" value="0.7"/></bsdf>',
     "roughness"),
    ('<bsdf type="roughplastic" id="x"><float name="intIOR" value="1.0"/><float name="extIOR" value="1.0"/></bsdf>',
     "differ"),
])
def test_roughplastic_errors(tmp_path, bsdf, msg):
    with pytest.raises(Exception, match=msg):
        _load(tmp_path, bsdf)
