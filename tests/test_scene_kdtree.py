"""Host scene loading + SAH kd-tree: the tree must give the brute-force
closest hit for every ray (traversal restated from sahkdtree3.h:178-308),
including the test_kd.cpp chord workload through the bunny."""
import os

import numpy as np

import mtsg
from oracle import pyoracle as O
from conftest import SCENES


def chords(n, center, radius, seed):
    # test_kd.cpp:112-118: chords between two uniform points on a sphere
    rng = np.random.default_rng(seed)
    def sph(k):
        v = rng.normal(size=(k, 3))
        return v / np.linalg.norm(v, axis=1, keepdims=True)
    a = center + radius * sph(n)
    b = center + radius * sph(n)
    d = b - a
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = a
    rays[:, 3:6] = d
    rays[:, 6] = 0.0
    rays[:, 7] = np.inf
    return rays


def check_against_brute(scene, rays):
    t, u, v, prim = O.trace_closest(scene.desc, rays)
    tb, pb = O.trace_closest_brute(scene.desc, rays)
    hit = prim != 0xFFFFFFFF
    assert np.array_equal(hit, pb != 0xFFFFFFFF)
    # identical closest distance; primitive ids may differ only on exact ties
    assert np.array_equal(t[hit], tb[hit])
    return hit.mean()


def test_cbox_loads(cbox_small):
    i = cbox_small.info
    assert i.n_triangles == 24 and i.n_rects == 6 and i.n_emitters == 1
    assert i.film_w == 64 and i.film_h == 48 and i.spp == 8 and i.border == 2
    p = cbox_small.params()
    assert (p.max_depth, p.rr_depth, p.spp) == (-1, 5, 8)


def test_cbox_kdtree_matches_brute_force(cbox_small):
    rng = np.random.default_rng(3)
    n = 20000
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = rng.uniform(-0.95, 0.95, (n, 3))
    d = rng.normal(size=(n, 3))
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 6] = 1e-4     # Epsilon -> adaptive epsilon path (skdtree.cpp:126-129)
    rays[:, 7] = np.inf
    frac = check_against_brute(cbox_small, rays)
    assert frac > 0.5


def test_bunny_instances_flattened(bunny_small):
    i = bunny_small.info
    assert i.n_triangles == 15 * 69451 == 1041765
    assert i.n_rects == 2
    assert i.kd_max_depth <= 48


def test_bunny_kdtree_chords(bunny_small):
    # bounding sphere of one instance region; brute force over 1M triangles is
    # O(n * prims), so keep n small
    rays = chords(64, np.array([0.0, 0.45, 0.0]), 0.8, 7)
    frac = check_against_brute(bunny_small, rays)
    assert frac > 0.3


def test_shadow_queries_consistent(cbox_small):
    rng = np.random.default_rng(5)
    n = 5000
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = rng.uniform(-0.9, 0.9, (n, 3))
    d = rng.normal(size=(n, 3))
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 6] = 1e-4
    rays[:, 7] = rng.uniform(0.05, 2.0, n)
    occ = O.trace_shadow(cbox_small.desc, rays)
    t, _, _, prim = O.trace_closest(cbox_small.desc, rays)
    # a shadow ray is occluded iff a closest hit exists within [mint, maxt]
    # (the shadow variant drops the 1e-4 floor of the adaptive epsilon)
    closest = (prim != 0xFFFFFFFF)
    agree = (occ.astype(bool) == closest)
    assert agree.mean() > 0.999


def test_bad_scene_reports_error(tmp_path):
    p = tmp_path / "bad.xml"
    p.write_text('<scene version="0.5.0"><integrator type="bdpt"/></scene>')
    try:
        mtsg.Scene(str(p))
    except RuntimeError as e:
        assert "bdpt" in str(e)
    else:
        raise AssertionError("expected an error")


def test_microfacet_distribution_parsing(tmp_path):
    # MicrofacetDistribution(props) (microfacet.h:96-144): beckmann / ggx /
    # phong = as, anisotropic alphaU / alphaV, the alpha-vs-alphaU/V errors
    for d in ("as", "phong", "ggx", "beckmann"):
        s = mtsg.Scene(os.path.join(SCENES, "cbox_rough.xml"),
                       {"width": 16, "height": 16, "spp": 1, "dist": d, "alphaU": 0.1, "alphaV": 0.3})
        assert s.info.n_triangles == 24
    bad = tmp_path / "bad.xml"
    for body, msg in (('<string name="distribution" value="blinn"/>', "invalid microfacet distribution"),
                      ('<float name="alpha" value="0.1"/><float name="alphaU" value="0.1"/>', "either 'alpha' or"),
                      ('<float name="alphaU" value="0.1"/>', "both 'alphaU' and 'alphaV'")):
        bad.write_text('<scene version="0.5.0"><shape type="cube"><bsdf type="roughconductor">'
                       + body + '</bsdf></shape></scene>')
        try:
            mtsg.Scene(str(bad))
        except RuntimeError as e:
            assert msg in str(e), str(e)
        else:
            raise AssertionError("expected an error for " + body)


def _bsdfs(scene):
    """The scene descriptor's BSDF records (include/mtsg.h mtsg_bsdf)."""
    import ctypes as C
    from test_bsdf_chisquare import Bsdf
    P, U = C.c_void_p, C.c_uint32

    class Head(C.Structure):
        _fields_ = [("abi", U), ("nv", U), ("pos", P), ("nrm", P), ("ntri", U), ("tri_idx", P), ("dpdu", P),
                    ("nrects", U), ("rects", P), ("nshapes", U), ("shapes", P), ("nbsdfs", U), ("bsdfs", P)]
    h = C.cast(scene.desc, C.POINTER(Head)).contents
    return list(C.cast(h.bsdfs, C.POINTER(Bsdf))[:h.nbsdfs])


def test_smooth_material_records():
    s = mtsg.Scene(os.path.join(SCENES, "cbox_materials.xml"), {"width": 16, "height": 16, "spp": 1})
    b = _bsdfs(s)
    plastic = [x for x in b if x.type == 5]
    assert len(plastic) == 2
    for p in plastic:
        eta = p.ior_eta
        # fresnelDiffuseReflectance(1 / eta): the reference's own fit for
        # eta < 1 (Egan & Hilgeman, util.cpp:822-833) to its stated accuracy
        e = 1 / eta
        fit = -1.4399 * e * e + 0.7099 * e + 0.6681 + 0.0636 / e
        assert abs(p.fdr_int - fit) < 6e-3 * fit, (p.fdr_int, fit)
        lum = lambda v: v[0] * 0.212671 + v[1] * 0.715160 + v[2] * 0.072169
        assert abs(p.spec_sampling_weight - lum(p.spec_refl) / (lum(p.reflectance) + lum(p.spec_refl))) < 1e-6
    assert plastic[0].ior_eta == np.float32(1.49) / np.float32(1.000277) and plastic[1].nonlinear == 1
    cond = [x for x in b if x.type == 4]
    assert len(cond) == 1 and cond[0].smooth == 0
    two = [x for x in b if x.twosided]
    assert len(two) == 2 and all(t.ref_n_zero == 1 and t.smooth == 1 for t in two)
    # the two-BRDF panel: front red, back green
    panel = [t for t in two if b[t.back].reflectance[1] > 0.4][0]
    assert panel.reflectance[0] > 0.6


def test_energy_conservation_scaling(tmp_path):
    # BSDF::ensureEnergyConservation (bsdf.cpp:88-113): scale by 0.99 / max
    p = tmp_path / "e.xml"
    p.write_text('<scene version="0.5.0"><sensor type="perspective"><film type="hdrfilm">'
                 '<integer name="width" value="8"/><integer name="height" value="8"/></film></sensor>'
                 '<shape type="cube"><bsdf type="diffuse">'
                 '<rgb name="reflectance" value="2, 1, 0.5"/></bsdf></shape>'
                 '<shape type="rectangle"><emitter type="area"/></shape></scene>')
    r = list(_bsdfs(mtsg.Scene(str(p)))[0].reflectance)
    np.testing.assert_allclose(r, [0.99, 0.495, 0.2475], rtol=1e-6)


def test_leaf_size_default_and_mitsuba_tree():
    """The build stops at 4 primitives per leaf (GPU-tuned, host/scene.h);
    the Scene's kdStopPrims property (scene.cpp:64-65) = 6 gives Mitsuba's tree
    (gkdtree.h:738), which bench.py's CPU baseline traverses.  Both trees
    answer the same closest hits."""
    path = os.path.join(SCENES, "bunny15.xml")
    defs = {"width": 16, "height": 16, "spp": 1}
    tuned = mtsg.Scene(path, defs)
    mitsuba = mtsg.Scene(path, defs, scene_props={"kdStopPrims": 6})
    assert mitsuba.info.kd_leaves < tuned.info.kd_leaves
    assert mitsuba.info.kd_indices < tuned.info.kd_indices
    rays = chords(20000, np.array([0.0, 0.45, 0.0]), 3.2, 5)
    t0, _, _, p0 = O.trace_closest(tuned.desc, rays)
    t1, _, _, p1 = O.trace_closest(mitsuba.desc, rays)
    same = p0 == p1
    assert same.mean() > 0.999
    np.testing.assert_array_equal(t0[same], t1[same])


def test_bench_cpu_baseline_uses_mitsubas_tree(bunny_small):
    """bench.py times its CPU baseline on the tree Mitsuba would build
    (kdStopPrims 6, through the Scene's properties), not on the GPU-tuned one."""
    import bench
    m = bench.mitsuba_tree_scene(bunny_small)
    assert m.info.n_triangles == bunny_small.info.n_triangles
    assert m.info.kd_indices < bunny_small.info.kd_indices


def _with_scene_props(tmp_path, body):
    """cbox.xml with `body` (value elements) as <scene>-level children."""
    src = open(os.path.join(SCENES, "cbox.xml")).read()
    i = src.index(">", src.index("<scene")) + 1
    p = tmp_path / "cbox_kd.xml"
    p.write_text(src[:i] + body + src[i:])
    return str(p)


def test_scene_kd_properties_on_the_xml_route(tmp_path):
    """<scene>'s kd properties (Scene::Scene, scene.cpp:47-83) reach the build:
    kdStopPrims 12 makes fewer, larger leaves; the hits stay identical."""
    defs = {"width": 16, "height": 16, "spp": 1}
    base = mtsg.Scene(os.path.join(SCENES, "cbox.xml"), defs)
    big = mtsg.Scene(_with_scene_props(tmp_path, '<integer name="kdStopPrims" value="12"/>'
                                                 '<float name="kdTraversalCost" value="10"/>'
                                                 '<boolean name="kdRetract" value="false"/>'), defs)
    assert big.info.kd_leaves < base.info.kd_leaves
    rng = np.random.default_rng(11)
    n = 20000
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = rng.uniform(-0.95, 0.95, (n, 3))
    d = rng.normal(size=(n, 3))
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 6] = 1e-4
    rays[:, 7] = np.inf
    t0, _, _, p0 = O.trace_closest(base.desc, rays)
    t1, _, _, p1 = O.trace_closest(big.desc, rays)
    assert np.array_equal(p0 != 0xFFFFFFFF, p1 != 0xFFFFFFFF)
    np.testing.assert_array_equal(t0, t1)
    # the same through the Scene properties a plugin passes (mtsh_scene_load_props)
    via = mtsg.Scene(os.path.join(SCENES, "cbox.xml"), defs,
                     scene_props={"kdStopPrims": 12, "kdTraversalCost": 10.0, "kdRetract": False})
    assert via.digest() == big.digest()


def test_scene_kd_properties_are_checked(tmp_path):
    defs = {"width": 16, "height": 16, "spp": 1}
    for body, msg in (('<integer name="kdStopPrim" value="12"/>', "unknown scene property"),
                      ('<float name="kdStopPrims" value="12"/>', "must be of type integer"),
                      ('<integer name="kdMaxDepth" value="99"/>', "kdMaxDepth")):
        try:
            mtsg.Scene(_with_scene_props(tmp_path, body), defs)
        except RuntimeError as e:
            assert msg in str(e), str(e)
        else:
            raise AssertionError("expected an error for " + body)
