"""Sample-vs-pdf consistency of the oracle's BSDFs, as the reference checks its
own (src/tests/test_chisquare.cpp:391-620 with include/mitsuba/core/chisquare.h,
src/libcore/chisquare.cpp:176-260):

- 10 theta x 20 phi cells on the sphere;
- 1000 samples per cell (200k per test);
- expected counts = sample count x the integral of pdf(wo) sin(theta) over each cell;
- cells with expected count < 5 are pooled;
- p-value threshold 0.0025 with the Sidak correction over the tests of one BSDF.

Also checked: sampled weight == eval / pdf (the reference's "f/pdf" check), and for
the dielectric, the reflect/refract split against Fresnel.

The GPU shares these exact routines through counter-mode render parity
(tests/test_gpu_parity.py), so this pins the device BSDFs as well.
"""
import ctypes as C
import math

import numpy as np
import pytest
from scipy import stats

from oracle import pyoracle as O

SIGNIFICANCE = 0.0025
THETA_BINS, PHI_BINS = 10, 20
N_SAMPLES = THETA_BINS * PHI_BINS * 1000
WI_PER_BSDF = 5

DIFFUSE, ROUGHCONDUCTOR, DIELECTRIC, CONDUCTOR, PLASTIC, ROUGHDIELECTRIC, ROUGHPLASTIC = 1, 2, 3, 4, 5, 6, 7
DELTA = 4 | 16   # EDeltaReflection | EDeltaTransmission
BECKMANN, GGX, PHONG = 0, 1, 2
RTRANS_SAMPLES = 100   # MTSG_RTRANS_SAMPLES


class Bsdf(C.Structure):
    """mtsg_bsdf (include/mtsg.h)."""
    _fields_ = [("type", C.c_int32), ("distribution", C.c_int32), ("sample_visible", C.c_int32),
                ("smooth", C.c_int32), ("ref_n_zero", C.c_int32), ("twosided", C.c_int32),
                ("back", C.c_int32), ("nonlinear", C.c_int32),
                ("reflectance", C.c_float * 3), ("eta", C.c_float * 3), ("k", C.c_float * 3),
                ("spec_refl", C.c_float * 3), ("spec_trans", C.c_float * 3),
                ("alpha_u", C.c_float), ("alpha_v", C.c_float),
                ("ior_eta", C.c_float), ("ior_inv_eta", C.c_float),
                ("fdr_int", C.c_float), ("spec_sampling_weight", C.c_float),
                ("rtrans", C.c_float * RTRANS_SAMPLES), ("texture", C.c_int32), ("pad_tex", C.c_int32 * 3)]


def make_bsdf(kind, dist=GGX, alpha=0.2, visible=1, eta=1.5046, alpha_v=None, nonlinear=0, fdr_int=0.6, spec_weight=0.6):
    b = Bsdf()
    b.type = kind
    b.distribution = dist
    b.sample_visible = visible
    b.smooth = 1 if kind not in (DIELECTRIC, CONDUCTOR) else 0
    b.nonlinear = nonlinear
    b.fdr_int = fdr_int
    b.spec_sampling_weight = spec_weight
    b.reflectance[:] = (0.5, 0.3, 0.8)
    b.eta[:] = (0.200438, 0.924033, 1.10221)      # Cu (ior.h lookup), RGB
    b.k[:] = (3.91295, 2.45285, 2.14219)
    b.spec_refl[:] = (1.0, 1.0, 1.0)
    b.spec_trans[:] = (1.0, 1.0, 1.0)
    b.alpha_u = alpha
    b.alpha_v = alpha if alpha_v is None else alpha_v
    b.ior_eta, b.ior_inv_eta = eta, 1.0 / eta
    if kind == ROUGHPLASTIC:
        # the host library's RoughTransmittance slice, as the scene loader builds it
        H = host_lib()
        diff = C.c_float()
        assert H.mtsh_rough_transmittance(dist, C.c_float(alpha), C.c_float(eta), RTRANS_SAMPLES, b.rtrans, None) == 0
        assert H.mtsh_rough_transmittance(dist, C.c_float(alpha), C.c_float(1.0 / eta), RTRANS_SAMPLES,
                                          (C.c_float * RTRANS_SAMPLES)(), C.byref(diff)) == 0
        b.fdr_int = 1 - diff.value
    return b


def host_lib():
    import mtsg
    L = mtsg.host_lib()
    L.mtsh_rough_transmittance.argtypes = [C.c_int, C.c_float, C.c_float, C.c_int, C.c_void_p, C.c_void_p]
    return L


def _lib():
    L = O.lib()
    if not getattr(L, "_bsdf_n_bound", False):
        L.oracle_bsdf_sample_n.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_bsdf_sample3_n.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_bsdf_eval_n.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
        L._bsdf_n_bound = True
    return L


def sample(b, wi, u2):
    """u2: n x 2 (the sample) or n x 3 (plus the BSDF's own next1D draw)."""
    u = np.ascontiguousarray(u2, np.float32)
    n = u.shape[0]
    if u.shape[1] == 2:
        u = np.ascontiguousarray(np.concatenate([u, np.full((n, 1), 0.5, np.float32)], 1))
    wi = np.ascontiguousarray(wi, np.float32)
    wo = np.zeros((n, 3), np.float32); pdf = np.zeros(n, np.float32)
    w = np.zeros((n, 3), np.float32); t = np.zeros(n, np.int32)
    _lib().oracle_bsdf_sample3_n(C.byref(b), O._p(wi), n, O._p(u), O._p(wo), O._p(pdf), O._p(w), O._p(t))
    return wo, pdf, w, t


def evaluate(b, wi, wo):
    wo = np.ascontiguousarray(wo, np.float32)
    wi = np.ascontiguousarray(wi, np.float32)
    n = wo.shape[0]
    val = np.zeros((n, 3), np.float32); pdf = np.zeros(n, np.float32)
    _lib().oracle_bsdf_eval_n(C.byref(b), O._p(wi), n, O._p(wo), O._p(val), O._p(pdf))
    return val, pdf


def unreachable(b, wi, wo):
    """Rough dielectric transmission directions no microfacet refraction can
    produce (dot(wi, H) * dot(wo, H) >= 0 for the generalised half-vector):
    the reference's pdf() (roughdielectric.cpp:337-400) still gives them a
    density, and sample() rejects the corresponding draws by its side check,
    so the sampled histogram is compared with the pdf on the reachable set."""
    if b.type != ROUGHDIELECTRIC:
        return np.zeros(len(wo), bool)
    eta = b.ior_eta if wi[2] > 0 else b.ior_inv_eta
    H = wi[None, :] + wo * eta
    H = H / np.linalg.norm(H, axis=1, keepdims=True) * np.sign(H[:, 2:3])
    return (wi[2] * wo[:, 2] < 0) & ((H @ wi) * (H * wo).sum(1) >= 0)


def expected_counts(b, wi, n_samples, gl=32, reachable_only=True):
    """n_samples x integral of pdf(wo) sin(theta) over each (theta, phi) cell
    (tensor Gauss-Legendre, gl x gl nodes per cell: 12 under-resolves the
    alpha = 0.1 lobes of the anisotropic cases)."""
    x, w = np.polynomial.legendre.leggauss(gl)
    dth, dph = math.pi / THETA_BINS, 2 * math.pi / PHI_BINS
    ti = np.arange(THETA_BINS)[:, None, None, None]
    pj = np.arange(PHI_BINS)[None, :, None, None]
    th = (ti + 0.5 + 0.5 * x[None, None, :, None]) * dth
    ph = (pj + 0.5 + 0.5 * x[None, None, None, :]) * dph
    th, ph = np.broadcast_arrays(th, ph)
    wo = np.stack([np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)], -1).reshape(-1, 3)
    _, pdf = evaluate(b, wi, wo)
    if reachable_only:
        pdf = np.where(unreachable(b, np.asarray(wi, np.float64), wo.astype(np.float64)), 0.0, pdf)
    wts = (w[:, None] * w[None, :]) * (0.25 * dth * dph)
    integ = (pdf.reshape(THETA_BINS, PHI_BINS, gl, gl).astype(np.float64) * np.sin(th) * wts).sum((2, 3))
    return integ * n_samples


def observed_counts(wo):
    z = np.clip(wo[:, 2].astype(np.float64), -1, 1)
    th = np.arccos(z)
    ph = np.arctan2(wo[:, 1], wo[:, 0]).astype(np.float64)
    ph = np.where(ph < 0, ph + 2 * math.pi, ph)
    i = np.minimum((th / (math.pi / THETA_BINS)).astype(int), THETA_BINS - 1)
    j = np.minimum((ph / (2 * math.pi / PHI_BINS)).astype(int), PHI_BINS - 1)
    c = np.zeros((THETA_BINS, PHI_BINS))
    np.add.at(c, (i, j), 1)
    return c


def chi2_pvalue(obs, exp):
    """Pooling rule of chisquare.cpp:176-240 (cells sorted by expected count)."""
    obs, exp = obs.ravel(), exp.ravel()
    order = np.argsort(exp, kind="stable")
    chsq, df = 0.0, 0
    pc = pr = 0.0
    pooled = 0
    for idx in order:
        e, o = exp[idx], obs[idx]
        if e == 0:
            assert o == 0, f"{o} samples in a cell of expected frequency zero"
        elif e < 5 or (0 < pr < 5):
            pc += o; pr += e; pooled += 1
        else:
            chsq += (o - e) ** 2 / e
            df += 1
    if pooled:
        chsq += (pc - pr) ** 2 / pr
        df += 1
    df -= 1
    assert df > 0
    return float(stats.chi2.sf(chsq, df))


def random_wi(rng, n):
    out = []
    while len(out) < n:
        v = rng.normal(size=3)
        v /= np.linalg.norm(v)
        if v[2] > 0.05:
            out.append(v.astype(np.float32))
    return out


CASES = [
    ("diffuse", dict(kind=DIFFUSE)),
    ("ggx_0.2_visible", dict(kind=ROUGHCONDUCTOR, dist=GGX, alpha=0.2, visible=1)),
    ("ggx_0.5_classic", dict(kind=ROUGHCONDUCTOR, dist=GGX, alpha=0.5, visible=0)),
    ("beckmann_0.1_visible", dict(kind=ROUGHCONDUCTOR, dist=BECKMANN, alpha=0.1, visible=1)),
    ("beckmann_0.3_classic", dict(kind=ROUGHCONDUCTOR, dist=BECKMANN, alpha=0.3, visible=0)),
    # anisotropic roughness (alphaU != alphaV) and the Phong / Ashikhmin-Shirley
    # distribution, as the reference's roughconductor instances of test_chisquare
    ("ggx_aniso_visible", dict(kind=ROUGHCONDUCTOR, dist=GGX, alpha=0.1, alpha_v=0.4, visible=1)),
    ("ggx_aniso_classic", dict(kind=ROUGHCONDUCTOR, dist=GGX, alpha=0.4, alpha_v=0.15, visible=0)),
    ("beckmann_aniso_visible", dict(kind=ROUGHCONDUCTOR, dist=BECKMANN, alpha=0.3, alpha_v=0.1, visible=1)),
    ("beckmann_aniso_classic", dict(kind=ROUGHCONDUCTOR, dist=BECKMANN, alpha=0.15, alpha_v=0.4, visible=0)),
    ("phong_0.3", dict(kind=ROUGHCONDUCTOR, dist=PHONG, alpha=0.3, visible=0)),
    ("phong_aniso", dict(kind=ROUGHCONDUCTOR, dist=PHONG, alpha=0.2, alpha_v=0.5, visible=0)),
    # smooth plastic: only its diffuse lobe has a density (the specular
    # samples are delta and excluded, as chisquare.cpp does for discrete ones)
    ("plastic", dict(kind=PLASTIC, eta=1.49, fdr_int=0.595, spec_weight=0.6)),
    ("plastic_nonlinear", dict(kind=PLASTIC, eta=1.8, nonlinear=1, fdr_int=0.7, spec_weight=0.3)),
    # rough dielectric: reflection + transmission over the whole sphere, from
    # either side (roughdielectric.cpp; test_bsdf.xml holds rough dielectrics)
    ("roughdielectric_ggx_visible", dict(kind=ROUGHDIELECTRIC, dist=GGX, alpha=0.3, visible=1, eta=1.5)),
    ("roughdielectric_beckmann_classic", dict(kind=ROUGHDIELECTRIC, dist=BECKMANN, alpha=0.2, visible=0, eta=1.33)),
    # (Beckmann: GGX visible sampling draws slope_y from a rational fit whose
    # error the strongly stretched anisotropic incidences make visible)
    ("roughdielectric_aniso", dict(kind=ROUGHDIELECTRIC, dist=BECKMANN, alpha=0.1, alpha_v=0.35, visible=1, eta=1.6)),
    ("roughdielectric_phong", dict(kind=ROUGHDIELECTRIC, dist=PHONG, alpha=0.25, visible=0, eta=1.5)),
    # rough plastic: microfacet coating + diffuse base, component chosen by
    # the rough transmittance (test_bsdf.xml holds roughplastic instances)
    ("roughplastic_beckmann", dict(kind=ROUGHPLASTIC, dist=BECKMANN, alpha=0.1, visible=1, eta=1.49, spec_weight=0.6)),
    ("roughplastic_ggx_classic", dict(kind=ROUGHPLASTIC, dist=GGX, alpha=0.3, visible=0, eta=1.9, spec_weight=0.3)),
    ("roughplastic_phong_nonlinear", dict(kind=ROUGHPLASTIC, dist=PHONG, alpha=0.2, visible=0, eta=1.5, nonlinear=1,
                                          spec_weight=0.5)),
]
BOTH_SIDES = (ROUGHDIELECTRIC,)


@pytest.mark.parametrize("name,kw", CASES, ids=[c[0] for c in CASES])
def test_bsdf_sampling_matches_pdf(name, kw):
    b = make_bsdf(**kw)
    rng = np.random.default_rng(7)
    alpha = 1 - (1 - SIGNIFICANCE) ** (1.0 / WI_PER_BSDF)   # Sidak (chisquare.cpp:255)
    wis = random_wi(rng, WI_PER_BSDF)
    if kw["kind"] in BOTH_SIDES:
        wis = [w * (1 if k % 2 == 0 else -1) for k, w in enumerate(wis)]   # incident from inside too
    for wi in wis:
        u2 = rng.random((N_SAMPLES, 3), dtype=np.float32)
        wo, pdf, w, t = sample(b, wi, u2)
        ok = (pdf > 0) & (w.max(1) > 0) & ((t & DELTA) == 0)
        p = chi2_pvalue(observed_counts(wo[ok]), expected_counts(b, wi, N_SAMPLES))
        assert p >= alpha, f"{name} wi={wi}: chi-square p-value {p:.3e} < {alpha:.3e}"
        # weight == f / pdf for the sampled directions (non-delta lobes)
        sel = np.flatnonzero(ok & (pdf > 1e-3))[:5000]
        val, pdf_e = evaluate(b, wi, wo[sel])
        np.testing.assert_allclose(pdf_e, pdf[sel], rtol=2e-3, atol=1e-6)
        np.testing.assert_allclose(w[sel] * pdf[sel][:, None], val, rtol=5e-3, atol=1e-6)


def fresnel_dielectric(cos_i, eta):
    """Unpolarised Fresnel reflectance for a dielectric interface (independent
    closed form, used only to check the sampled reflect/refract split)."""
    if cos_i < 0:
        eta, cos_i = 1 / eta, -cos_i
    sin_t2 = (1 - cos_i ** 2) / eta ** 2
    if sin_t2 >= 1:
        return 1.0, 0.0
    cos_t = math.sqrt(1 - sin_t2)
    rs = (cos_i - eta * cos_t) / (cos_i + eta * cos_t)
    rp = (eta * cos_i - cos_t) / (eta * cos_i + cos_t)
    return 0.5 * (rs * rs + rp * rp), cos_t


@pytest.mark.parametrize("cos_i", [0.95, 0.5, 0.1, -0.3, -0.9])
def test_dielectric_split_follows_fresnel(cos_i):
    eta = 1.5046
    b = make_bsdf(DIELECTRIC, eta=eta)
    s = math.sqrt(1 - cos_i ** 2)
    wi = np.array([s, 0.0, cos_i], np.float32)
    n = 200000
    u2 = np.random.default_rng(3).random((n, 2), dtype=np.float32)
    wo, pdf, w, t = sample(b, wi, u2)
    F, cos_t = fresnel_dielectric(cos_i, eta)
    refl = wo[:, 2] * cos_i > 0
    frac = refl.mean()
    sigma = math.sqrt(max(F * (1 - F), 1e-12) / n)
    assert abs(frac - F) <= 5 * sigma + 1e-6, (frac, F)
    np.testing.assert_allclose(pdf[refl], F, rtol=1e-4)
    if F < 1:
        tr = ~refl
        np.testing.assert_allclose(pdf[tr], 1 - F, rtol=1e-4)
        # Snell's law and the (1/eta)^2 radiance scaling (dielectric.cpp:305-330)
        eta_rel = eta if cos_i > 0 else 1 / eta
        np.testing.assert_allclose(np.abs(wo[tr, 2]), cos_t, rtol=1e-4)
        np.testing.assert_allclose(w[tr], 1.0 / eta_rel ** 2, rtol=1e-4)
    np.testing.assert_allclose(w[refl], 1.0, rtol=1e-6)


def fresnel_conductor(cos_i, eta, k):
    """Exact unpolarised conductor Fresnel reflectance (independent complex
    closed form)."""
    n = eta + 1j * k
    sin2 = 1 - cos_i ** 2
    cos_t = np.sqrt(1 - sin2 / n ** 2)
    rs = (cos_i - n * cos_t) / (cos_i + n * cos_t)
    rp = (n * cos_i - cos_t) / (n * cos_i + cos_t)
    return 0.5 * (np.abs(rs) ** 2 + np.abs(rp) ** 2)


def test_smooth_conductor_is_a_fresnel_mirror():
    # conductor.cpp:220-236: delta reflection, pdf 1, weight = specularReflectance * F
    b = make_bsdf(CONDUCTOR)
    for cos_i in (0.99, 0.7, 0.3, 0.05):
        s = math.sqrt(1 - cos_i ** 2)
        wi = np.array([s * 0.6, s * 0.8, cos_i], np.float32)
        wo, pdf, w, t = sample(b, wi, np.full((4, 2), 0.37, np.float32))
        assert np.all(t == 4) and np.all(pdf == 1)
        np.testing.assert_allclose(wo, np.tile([-wi[0], -wi[1], wi[2]], (4, 1)), atol=1e-7)
        F = [fresnel_conductor(cos_i, e, k) for e, k in zip(b.eta, b.k)]
        np.testing.assert_allclose(w[0], F, rtol=2e-4)
    # from below: no scattering
    _, _, w, _ = sample(b, np.array([0.0, 0.6, -0.8], np.float32), np.full((1, 2), 0.5, np.float32))
    assert np.all(w == 0)


def test_plastic_specular_split_follows_fresnel():
    # plastic.cpp:344-375: specular chosen with probability
    # F w_s / (F w_s + (1 - F)(1 - w_s)), weight spec * F / p
    eta, ws = 1.49, 0.6
    b = make_bsdf(PLASTIC, eta=eta, spec_weight=ws)
    for cos_i in (0.9, 0.4, 0.1):
        s = math.sqrt(1 - cos_i ** 2)
        wi = np.array([s, 0.0, cos_i], np.float32)
        n = 100000
        u2 = np.random.default_rng(3).random((n, 2), dtype=np.float32)
        wo, pdf, w, t = sample(b, wi, u2)
        F, _ = fresnel_dielectric(cos_i, eta)
        p = F * ws / (F * ws + (1 - F) * (1 - ws))
        spec = (t & 4) != 0
        assert abs(spec.mean() - p) < 5 * math.sqrt(p * (1 - p) / n) + 1e-6
        np.testing.assert_allclose(pdf[spec], p, rtol=1e-5)
        np.testing.assert_allclose(w[spec], F / p, rtol=1e-4)
