"""GPU parity: the HIP wavefront path (through the C-ABI) against the CPU
oracle on identical inputs.  Bars (DESIGN.md "Parity"):
  * traversal: identical closest primitive except exact-distance ties,
    t/u/v within 1e-4 relative;
  * render (counter-mode RNG, identical random numbers per pixel/sample/
    dimension): mean per-pixel L1 of the developed image < 1e-3 of the
    mean radiance, filter-weight channel within 1e-5 relative."""
import os

import numpy as np
import pytest

import mtsg
from oracle import pyoracle as O
from conftest import SCENES

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_cbox(cbox_small):
    g = mtsg.GPUScene(cbox_small, 0)
    yield g
    g.close()


@pytest.fixture(scope="module")
def gpu_bunny(bunny_small):
    g = mtsg.GPUScene(bunny_small, 0)
    yield g
    g.close()


def random_rays(n, lo, hi, seed, mint=1e-4):
    rng = np.random.default_rng(seed)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = rng.uniform(lo, hi, (n, 3))
    d = rng.normal(size=(n, 3))
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 6] = mint
    rays[:, 7] = np.inf
    return rays


def compare_closest(scene, g, rays):
    t0, u0, v0, p0 = O.trace_closest(scene.desc, rays)
    t1, u1, v1, p1 = g.trace_closest(rays)
    hit0, hit1 = p0 != 0xFFFFFFFF, p1 != 0xFFFFFFFF
    assert (hit0 != hit1).mean() < 1e-4
    both = hit0 & hit1
    same = both & (p0 == p1)
    # differing primitives only on (near-)ties of the hit distance
    diff = both & (p0 != p1)
    assert np.all(np.abs(t0[diff] - t1[diff]) <= 1e-4 * np.abs(t0[diff]) + 1e-6)
    assert same.sum() >= 0.999 * both.sum()
    np.testing.assert_allclose(t1[same], t0[same], rtol=1e-4, atol=1e-6)
    # the triangle/rectangle tests run without FMA contraction on both sides:
    # same primitive => bit-identical distance and barycentrics
    np.testing.assert_array_equal(t1[same], t0[same])
    np.testing.assert_array_equal(u1[same], u0[same])
    np.testing.assert_array_equal(v1[same], v0[same])
    return both.mean()


def test_device_visible():
    assert mtsg.device_lib().mtsg_device_count() >= 1


def test_trace_closest_cbox(cbox_small, gpu_cbox):
    assert compare_closest(cbox_small, gpu_cbox, random_rays(100000, -0.95, 0.95, 1)) > 0.5


def test_trace_closest_bunny_chords(bunny_small, gpu_bunny):
    # kdbench / test_kd.cpp style incoherent chords through the instanced bunnies
    rng = np.random.default_rng(2)
    n = 200000
    def sph(k):
        v = rng.normal(size=(k, 3))
        return v / np.linalg.norm(v, axis=1, keepdims=True)
    c = np.array([0.0, 0.45, 0.0])
    a = c + 3.2 * sph(n)
    b = c + 3.2 * sph(n)
    d = b - a
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = a; rays[:, 3:6] = d; rays[:, 6] = 0.0; rays[:, 7] = np.inf
    assert compare_closest(bunny_small, gpu_bunny, rays) > 0.2


def test_trace_shadow(cbox_small, gpu_cbox, bunny_small, gpu_bunny):
    for scene, g, lo, hi in ((cbox_small, gpu_cbox, -0.9, 0.9), (bunny_small, gpu_bunny, -2.5, 2.5)):
        rays = random_rays(100000, lo, hi, 11)
        rays[:, 7] = np.random.default_rng(12).uniform(0.05, 3.0, len(rays))
        o0 = O.trace_shadow(scene.desc, rays)
        o1 = g.trace_shadow(rays)
        assert (o0 != o1).mean() < 1e-4


def render_pair(scene, g, **over):
    p = scene.params(**over)
    b = scene.border
    img_c, _ = O.render(scene.desc, p, b, rng=O.RNG_COUNTER)
    img_g = g.render(p, b)
    return p, img_c, img_g


def check_render(img_c, img_g):
    w_c, w_g = img_c[..., 4], img_g[..., 4]
    np.testing.assert_allclose(w_g, w_c, rtol=1e-5, atol=1e-5)
    rgb_c, rgb_g = mtsg.develop(img_c), mtsg.develop(img_g)
    l1 = np.abs(rgb_c - rgb_g).mean()
    mean = rgb_c.mean()
    assert mean > 0
    assert l1 < 1e-3 * max(mean, 1e-3) + 1e-6, (l1, mean)
    return l1, mean


def test_render_cbox_parity(cbox_small, gpu_cbox):
    _, c, g = render_pair(cbox_small, gpu_cbox)
    check_render(c, g)


def test_render_cbox_maxdepth_and_hide_emitters(cbox_small, gpu_cbox):
    for over in ({"max_depth": 1}, {"max_depth": 2}, {"max_depth": 8, "hide_emitters": 1},
                 {"max_depth": 3, "strict_normals": 1}, {"rr_depth": 1}):
        _, c, g = render_pair(cbox_small, gpu_cbox, **over)
        check_render(c, g)


def test_render_tile_and_seed(cbox_small, gpu_cbox):
    # a ragged sub-rectangle (not a multiple of the 16x16 splat tile)
    _, c, g = render_pair(cbox_small, gpu_cbox, tile_x=5, tile_y=7, tile_w=37, tile_h=19, seed=3)
    check_render(c, g)


def test_render_bunny_roughconductor_parity(bunny_small, gpu_bunny):
    _, c, g = render_pair(bunny_small, gpu_bunny)
    check_render(c, g)


def test_tiling_is_additive(cbox_small, gpu_cbox):
    # film tiled over 2 "GPUs" (two calls) + additive border merge == one call
    p = cbox_small.params()
    b = cbox_small.border
    full = gpu_cbox.render(p, b)
    left = gpu_cbox.render(cbox_small.params(tile_w=32), b)
    right = gpu_cbox.render(cbox_small.params(tile_x=32, tile_w=32), b)
    merged = np.zeros_like(full)
    merged[:, 0:32 + 2 * b] += left
    merged[:, 32:64 + 2 * b] += right
    np.testing.assert_allclose(merged, full, rtol=2e-5, atol=2e-5)


def test_staggered_lanes_are_bit_identical(cbox_small):
    # the multi-lane render path (MTSG_OPT_LANES batches on their own streams,
    # MTSG_OPT_STAGGER bounces apart) renders the same samples as one lane
    p = cbox_small.params()
    b = cbox_small.border
    g1 = mtsg.GPUScene(cbox_small, 0)
    ref = g1.render(p, b)
    g1.close()
    g3 = mtsg.GPUScene(cbox_small, 0)
    g3.set_option(mtsg.MTSG_OPT_LANES, 3)
    g3.set_option(mtsg.MTSG_OPT_STAGGER, 2)
    g3.set_batch_paths(16 * 16 * 4 * 4)
    img = g3.render(p, b)
    g3.close()
    np.testing.assert_allclose(img, ref, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("tail", ["default", "per-bounce", "late-tail"])
@pytest.mark.parametrize("name", ["cbox.xml", "bunny15.xml", "env_glass.xml", "cbox_glass.xml"])
def test_material_kernels_match_the_generic_kernel(name, tail):
    # k_shade<.., MATS> and k_finish<.., MATS> hold only the scene's material
    # classes (diffuse / GGX roughconductor / dielectric): the same
    # arithmetic as the kernels with every class, so every sample's radiance is
    # bit-identical (the film itself sums samples with float atomics in no fixed
    # order).  tail: the small frame's paths go to the tail kernel after bounce 0
    # (default threshold), never (per-bounce launches only), or once fewer than
    # 4096 remain (per-bounce launches first, then the tail kernel)
    scene = mtsg.Scene(os.path.join(SCENES, name), {"width": 64, "height": 48, "spp": 8})
    p = scene.params()
    g = mtsg.GPUScene(scene, 0)
    if tail != "default":
        g.set_finish_paths(0 if tail == "per-bounce" else 4096)
    spec = g.render_samples(p)
    st = g.stats()
    if tail != "late-tail":
        assert (st.launches_finish > 0) == (tail == "default"), st.launches_finish
    g.set_option(mtsg.MTSG_OPT_SHADE_GENERIC, 1)
    gen = g.render_samples(p)
    g.close()
    assert np.array_equal(spec, gen, equal_nan=True), f"{name}: max |diff| {np.nanmax(np.abs(spec - gen))}"


@pytest.mark.parametrize("name", ["bunny15.xml", "env_glass.xml", "cbox_glass.xml"])
def test_tail_shading_threshold_does_not_change_samples(name):
    # the tail kernel shades a wave's waiting lanes once 16 of them wait (the
    # default) or as soon as one does (MTSG_OPT_FINISH_SHADE_MIN 1, the default
    # through round 5): which iteration shades a path changes nothing in its
    # arithmetic, so every sample is bit-identical
    scene = mtsg.Scene(os.path.join(SCENES, name), {"width": 64, "height": 48, "spp": 8})
    p = scene.params()
    g = mtsg.GPUScene(scene, 0)
    a = g.render_samples(p)
    assert g.stats().launches_finish > 0
    g.set_option(mtsg.MTSG_OPT_FINISH_SHADE_MIN, 1)
    b = g.render_samples(p)
    g.set_option(mtsg.MTSG_OPT_FINISH_SHADE_MIN, 64)
    c = g.render_samples(p)
    g.close()
    assert np.array_equal(a, b, equal_nan=True), f"{name}: max |diff| {np.nanmax(np.abs(a - b))}"
    assert np.array_equal(a, c, equal_nan=True), f"{name}: max |diff| {np.nanmax(np.abs(a - c))}"


@pytest.mark.parametrize("name", ["env_glass.xml", "cbox_textured.xml"])
def test_recomputed_camera_differentials_match_stored_ones(name):
    # an environment scene's camera ray that misses recomputes its ray
    # differentials at bounce 0 from the camera (DevScene::cam_env_diffs)
    # instead of reading them from the path state (MTSG_OPT_CAMERA_DIFFS 1, the
    # layout through round 5): the same arithmetic, so every sample's radiance
    # is bit-identical.  cbox_textured.xml (filtered textures: always stored)
    # must not change either
    scene = mtsg.Scene(os.path.join(SCENES, name), {"width": 80, "height": 64, "spp": 8})
    p = scene.params()
    g = mtsg.GPUScene(scene, 0)
    rec = g.render_samples(p)
    g.set_option(mtsg.MTSG_OPT_CAMERA_DIFFS, 1)
    stored = g.render_samples(p)
    g.close()
    assert np.isfinite(rec).all()
    assert np.array_equal(rec, stored, equal_nan=True), f"{name}: max |diff| {np.nanmax(np.abs(rec - stored))}"


@pytest.mark.parametrize("name", ["cbox.xml", "bunny15.xml"])
def test_refill_width_does_not_change_samples(name):
    # a traversal wave refills its idle lanes from the work list at 16 idle
    # lanes (default) or 32 (MTSG_OPT_TRACE_REFILL): when a ray is started
    # does not change its hit, so every sample is bit-identical
    scene = mtsg.Scene(os.path.join(SCENES, name), {"width": 80, "height": 64, "spp": 8})
    p = scene.params()
    g = mtsg.GPUScene(scene, 0)
    g.set_finish_paths(0)   # every bounce through the per-bounce traversal launches
    a = g.render_samples(p)
    g.set_option(mtsg.MTSG_OPT_TRACE_REFILL, 32)
    b = g.render_samples(p)
    g.close()
    assert np.array_equal(a, b, equal_nan=True), f"{name}: max |diff| {np.nanmax(np.abs(a - b))}"


@pytest.mark.parametrize("name", ["cbox.xml", "bunny15.xml", "env_glass.xml"])
def test_ray_order_does_not_change_samples(name):
    # the traversal takes bounce rays in direction-sorted windows
    # (MTSG_OPT_RAY_ORDER 1, k_sortwin) or in append order (0): the hit of a
    # ray does not depend on when it is traced, so every sample is bit-identical
    scene = mtsg.Scene(os.path.join(SCENES, name), {"width": 80, "height": 64, "spp": 8})
    p = scene.params()
    g = mtsg.GPUScene(scene, 0)
    g.set_option(mtsg.MTSG_OPT_RAY_ORDER, 1)
    sorted_ = g.render_samples(p)
    g.set_option(mtsg.MTSG_OPT_RAY_ORDER, 0)
    plain = g.render_samples(p)
    g.close()
    assert np.array_equal(sorted_, plain, equal_nan=True), f"{name}: max |diff| {np.nanmax(np.abs(sorted_ - plain))}"


def test_set_option_rejects_unknown_keys_and_values(cbox_small):
    g = mtsg.GPUScene(cbox_small, 0)
    for key, value in ((99, 1), (mtsg.MTSG_OPT_LANES, 0), (mtsg.MTSG_OPT_TRACE_REFILL, 20), (mtsg.MTSG_OPT_CAMERA_DIFFS, 2)):
        with pytest.raises(RuntimeError):
            g.set_option(key, value)
    g.close()


def test_dielectric_scene_parity():
    # smooth dielectric: delta BSDF, no NEE, MIS weight 1 on emitter hits, eta in RR
    scene = mtsg.Scene(os.path.join(SCENES, "cbox_glass.xml"), {"width": 48, "height": 48, "spp": 8})
    g = mtsg.GPUScene(scene, 0)
    _, c, gi = render_pair(scene, g)
    check_render(c, gi)
    g.close()


@pytest.fixture(scope="module")
def env_scene():
    scene = mtsg.Scene(os.path.join(SCENES, "env_glass.xml"), {"width": 64, "height": 36, "spp": 8, "maxDepth": 16})
    g = mtsg.GPUScene(scene, 0)
    yield scene, g
    g.close()


def test_envmap_scene_parity(env_scene):
    # environment emitter (C5): EWA lookups of primary misses, bilinear
    # lookups + MIS of BSDF-sampled misses, importance-sampled NEE with shadow
    # rays to the bounding sphere; dielectric + rough conductor + diffuse.
    # Device atan2f/acosf/sincosf differ from glibc by an ulp, so the bar is
    # the same image-level L1 as the other scenes.
    scene, g = env_scene
    _, c, gi = render_pair(scene, g)
    check_render(c, gi)


def test_envmap_hide_emitters_and_depth(env_scene):
    scene, g = env_scene
    for over in ({"hide_emitters": 1}, {"max_depth": 2}, {"max_depth": 64, "rr_depth": 2}):
        _, c, gi = render_pair(scene, g, **over)
        check_render(c, gi)


def test_envmap_lookup_parity(env_scene):
    # bilinear (BSDF-sampled rays) and EWA (camera rays with differentials)
    # lookups on the device vs the oracle, for footprints from sub-texel to
    # several MIP levels
    import ctypes as C
    scene, g = env_scene
    rng = np.random.default_rng(5)
    n = 4096
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    s = (10 ** rng.uniform(-3.5, -1, size=(n, 1))).astype(np.float32)
    t1 = np.cross(d, rng.normal(size=(n, 3))).astype(np.float32)
    t2 = np.cross(d, t1).astype(np.float32)
    rx = (d + s * t1).astype(np.float32)
    ry = (d + 0.6 * s * t2).astype(np.float32)
    L = O.lib()
    L.oracle_env_eval_n.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    for args in ((None, None), (rx, ry)):
        ref = np.zeros((n, 3), np.float32)
        px = None if args[0] is None else O._p(args[0])
        py = None if args[1] is None else O._p(args[1])
        L.oracle_env_eval_n(scene.desc, n, O._p(d), px, py, O._p(ref))
        got = g.env_eval(d, *args)
        # device atan2f / acosf differ from glibc's by an ulp; on the
        # reference's high-contrast envmap.exr a texel-coordinate ulp moves a
        # lookup by up to ~1e-3 relative: 99.9% within 2e-4, all within 2e-3
        rel = np.abs(got - ref) / (np.abs(ref) + 1e-6)
        assert (rel <= 2e-4).mean() >= 0.999, (rel > 2e-4).mean()
        np.testing.assert_allclose(got, ref, rtol=2e-3, atol=1e-6)


ROUGH_VARIANTS = [
    dict(dist="ggx", alphaU=0.05, alphaV=0.3),                           # anisotropic, visible normals
    dict(dist="beckmann", alphaU=0.3, alphaV=0.08),
    dict(dist="ggx", alphaU=0.4, alphaV=0.15, sampleVisible="false"),   # anisotropic sampleAll
    dict(dist="as", alphaU=0.1, alphaV=0.3),                             # test_bsdf.xml's Ashikhmin-Shirley instance
    dict(dist="phong", alphaU=0.25, alphaV=0.25),
]


@pytest.mark.parametrize("defs", ROUGH_VARIANTS, ids=lambda d: "-".join(str(v) for v in d.values()))
def test_rough_conductor_variants_parity(defs):
    # roughconductor with anisotropic roughness and the Phong / A&S distribution
    # (microfacet.h: eval, smithG1 with projectRoughness, sampleAll, sampleVisible)
    scene = mtsg.Scene(os.path.join(SCENES, "cbox_rough.xml"), dict(defs, width=48, height=48, spp=8))
    g = mtsg.GPUScene(scene, 0)
    _, c, gi = render_pair(scene, g)
    check_render(c, gi)
    g.close()
    pp = per_pixel_l1(c, gi, scene.border)
    print(f"cbox_rough {defs}: per-pixel max {pp.max():.2e}")
    assert pp.max() < 1e-3


def per_pixel_l1(img_c, img_g, border):
    b = border
    return np.abs(mtsg.develop(img_g[b:-b, b:-b]) - mtsg.develop(img_c[b:-b, b:-b])).mean(-1)


def test_default_roughconductor_per_pixel():
    """Mitsuba's default roughconductor (Beckmann, alpha 0.1, visible normals:
    microfacet.h:99-146, 573-697), a rougher Beckmann and a Phong lobe, whose
    sampling and evaluation call powf: with glibc's powf restated on the
    device (glibc_mathf.h) every pixel agrees with the oracle to < 1e-3 at
    64 spp, not only the image mean."""
    scene = mtsg.Scene(os.path.join(SCENES, "cbox_beckmann.xml"), {"width": 96, "height": 96, "spp": 64})
    g = mtsg.GPUScene(scene, 0)
    try:
        _, c, gi = render_pair(scene, g)
    finally:
        g.close()
    l1, mean = check_render(c, gi)
    pp = per_pixel_l1(c, gi, scene.border)
    print(f"cbox_beckmann 96x96x64: L1 {l1:.2e} of mean {mean:.4f}; per-pixel p99 {np.percentile(pp, 99):.2e} "
          f"max {pp.max():.2e}, {(pp > 1e-3).mean():.4%} above 1e-3")
    assert pp.max() < 1e-3


def test_smooth_materials_scene_parity():
    # plastic (linear and nonlinear), smooth conductor, twosided with one and
    # with two nested BRDFs (back side seen by the camera)
    scene = mtsg.Scene(os.path.join(SCENES, "cbox_materials.xml"), {"width": 48, "height": 48, "spp": 8})
    g = mtsg.GPUScene(scene, 0)
    _, c, gi = render_pair(scene, g)
    check_render(c, gi)
    _, c, gi = render_pair(scene, g, max_depth=3, strict_normals=1)
    check_render(c, gi)
    g.close()


def test_roughplastic_scene_parity():
    # roughplastic: Beckmann / GGX (visible and classic) / Phong coatings,
    # nonlinear, twosided front and back; rough transmittance slices and the
    # sample.y component split (roughplastic.cpp:387-455)
    scene = mtsg.Scene(os.path.join(SCENES, "cbox_roughplastic.xml"), {"width": 48, "height": 48, "spp": 8})
    g = mtsg.GPUScene(scene, 0)
    _, c, gi = render_pair(scene, g)
    check_render(c, gi)
    pp = per_pixel_l1(c, gi, scene.border)   # the rtrans lookup's powf(cos, 0.25) is glibc's
    _, c, gi = render_pair(scene, g, max_depth=3, strict_normals=1)
    check_render(c, gi)
    g.close()
    print(f"cbox_roughplastic: per-pixel max {pp.max():.2e}")
    assert pp.max() < 1e-3


@pytest.mark.parametrize("defs", [dict(dist="ggx", alpha=0.2), dict(dist="beckmann", alpha=0.35, sampleVisible="false")],
                         ids=["ggx-visible", "beckmann-classic"])
def test_rough_dielectric_parity(defs):
    # roughdielectric: glossy reflection + transmission, the extra next1D draw
    # of the reflect/refract choice, eta tracked through Russian roulette
    scene = mtsg.Scene(os.path.join(SCENES, "cbox_roughglass.xml"), dict(defs, width=48, height=48, spp=8))
    g = mtsg.GPUScene(scene, 0)
    _, c, gi = render_pair(scene, g)
    check_render(c, gi)
    g.close()


def test_c3_full_frame_parity():
    # the headline frame (C3: 15 bunnies, 1,041,765 triangles, roughconductor,
    # 1280x720, maxDepth 8) at 2 spp through the production render entry,
    # every pixel against the oracle (counter-mode RNG => identical samples)
    scene = mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 1280, "height": 720, "spp": 2})
    g = mtsg.GPUScene(scene, 0)
    p, c, gi = render_pair(scene, g)
    g.close()
    assert (p.tile_w, p.tile_h, p.max_depth) == (1280, 720, 8)
    l1, mean = check_render(c, gi)
    print(f"C3 1280x720x2spp: per-pixel L1 {l1:.3e}, mean {mean:.4f}, L1/mean {l1 / mean:.2e}")


def test_envmap_synthetic_sky_parity():
    # round 1's synthetic sky (tools/gen_envmap.py) as a second environment map
    scene = mtsg.Scene(os.path.join(SCENES, "env_glass.xml"),
                       {"width": 48, "height": 27, "spp": 8, "maxDepth": 16, "envmap": "sky512.pfm"})
    g = mtsg.GPUScene(scene, 0)
    _, c, gi = render_pair(scene, g)
    g.close()
    check_render(c, gi)


def test_coplanar_tie_policy():
    """Coplanar primitives: with -D glassY=-0.7 the glass box's bottom face
    lies on the floor (as the tall box's always does), so rays through the
    footprints meet a box triangle and the floor rectangle at exactly the
    same distance.  Mitsuba accepts a hit at t <= the best distance, in
    leaf order, skipping primitives still in its 8-entry mailbox
    (sahkdtree3.h:250-290), so the tie goes to the primitive tested last
    whose retest was not a mailbox hit; the GPU emulates the mailbox on
    ties (kernels.h mailbox_step), so the winner must be the oracle's, bit
    for bit -- from below the floor, from inside the boxes, from random
    points of the scene (ties on every coplanar face pair it has), and in
    a render of the dielectric scene with the box standing on the floor."""
    scene = mtsg.Scene(os.path.join(SCENES, "cbox_glass.xml"), {"width": 48, "height": 48, "spp": 8, "glassY": -0.7})
    b = scene.prim_bounds()
    flat = np.flatnonzero((b[:, 1] == -1.0) & (b[:, 4] == -1.0))
    assert flat.size >= 5   # two triangles of each box bottom + the floor
    rng = np.random.default_rng(17)
    rays = []
    for p in flat[:-1]:   # footprints of the box bottoms
        n = 4000
        x = rng.uniform(b[p, 0], b[p, 3], n)
        z = rng.uniform(b[p, 2], b[p, 5], n)
        for y0, dy in ((-1.0 - 0.25, 1.0), (-1.0 + 0.05, -1.0)):   # from below the floor, from inside the box
            r = np.zeros((n, 8), np.float32)
            r[:, 0], r[:, 1], r[:, 2] = x, y0, z
            d = np.stack([rng.normal(0, 0.05, n), np.full(n, dy), rng.normal(0, 0.05, n)], 1)
            r[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
            r[:, 6], r[:, 7] = 1e-4, np.inf
            rays.append(r)
    n_cop = sum(len(x) for x in rays)
    n = 100000
    r = np.zeros((n, 8), np.float32)
    r[:, :3] = rng.uniform(-1, 1, (n, 3))
    d = rng.normal(size=(n, 3))
    r[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    r[:, 6], r[:, 7] = 1e-4, np.inf
    rays.append(r)
    rays = np.concatenate(rays)
    g = mtsg.GPUScene(scene, 0)
    try:
        t0, u0, v0, p0 = O.trace_closest(scene.desc, rays)
        t1, u1, v1, p1 = g.trace_closest(rays)
        hit = p0 != 0xFFFFFFFF
        nt = scene.info.n_triangles
        ids = np.where(flat < nt, flat, 0x80000000 | (flat - nt)).astype(np.uint32)
        assert np.isin(p0[:n_cop][hit[:n_cop]], ids).mean() > 0.5    # the rays do meet the coplanar pairs
        np.testing.assert_array_equal(p1, p0)
        np.testing.assert_array_equal(t1, t0)
        np.testing.assert_array_equal(u1[hit], u0[hit])
        _, c, gi = render_pair(scene, g)
        check_render(c, gi)
    finally:
        g.close()
