"""The integrator-level entry points on the GPU: the multi-GPU render()
(mtsh_path_job_render / mtsh_path_render, include/mtsg_path.h, standing in for
SamplingIntegrator::render, src/librender/integrator.cpp:99-133), cancel()
(integrator.cpp:94-97) from a second thread, and the C4 film tiling on the C3
scene (tile shares merged by addition, imageblock.h:103-107)."""
import os
import threading
import time

import numpy as np
import pytest

import mtsg
from conftest import SCENES

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bunny_c3_small():
    # C3's scene (15 bunnies, 1,041,765 triangles) at a reduced frame
    return mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 320, "height": 180, "spp": 4})


@pytest.fixture(scope="module")
def gpu_c3(bunny_c3_small):
    g = mtsg.GPUScene(bunny_c3_small, 0)
    yield g
    g.close()


@pytest.mark.skipif(bool(os.environ.get("MTSG_LIB")),
                    reason="libmtsg_path.so links the default libmtsg.so, not the MTSG_LIB variant")
def test_path_render_matches_device_render(bunny_c3_small, gpu_c3):
    p = bunny_c3_small.params()
    b = bunny_c3_small.border
    ref = gpu_c3.render(p, b)
    for n in (1, 0):   # one GPU, all visible GPUs
        job = mtsg.PathJob(bunny_c3_small, n)
        rc, img, secs = job.render(p, b)
        assert rc == 0, job.last_error()
        assert secs > 0
        # the GPUs' blocks are summed on the host: equal up to float addition order
        np.testing.assert_allclose(img, ref, rtol=1e-5, atol=1e-6)
        job.close()


def test_path_render_composes_the_callers_tile_share(bunny_c3_small, gpu_c3):
    # a caller-supplied tile subset is kept (dealt over the job's GPUs), not overwritten
    b = bunny_c3_small.border
    p = bunny_c3_small.params(tile_stride=3, tile_offset=1)
    ref = gpu_c3.render(p, b)
    job = mtsg.PathJob(bunny_c3_small, 1)
    rc, img, _ = job.render(p, b)
    assert rc == 0, job.last_error()
    np.testing.assert_allclose(img, ref, rtol=1e-5, atol=1e-6)
    rc, _, _ = job.render(bunny_c3_small.params(tile_stride=3, tile_offset=3), b)
    assert rc == -1 and "tile_stride" in job.last_error()
    job.close()


def test_path_render_one_shot(bunny_c3_small, gpu_c3):
    import ctypes as C
    p = bunny_c3_small.params(spp=2)
    b = bunny_c3_small.border
    out = np.zeros((p.tile_h + 2 * b, p.tile_w + 2 * b, 5), np.float32)
    secs = C.c_double()
    rc = mtsg.path_lib().mtsh_path_render(C.c_void_p(bunny_c3_small._h), C.byref(p), 1,
                                          C.c_void_p(out.ctypes.data), C.byref(secs))
    assert rc == 0
    np.testing.assert_allclose(out, gpu_c3.render(p, b), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_c4_tile_shares_sum_to_the_full_frame(bunny_c3_small, gpu_c3, n):
    # config C4 on one GPU: the n ranks' tile shares (t % n == r) rendered one
    # after the other and summed equal the single-GPU frame (global RNG keys,
    # so the image does not depend on n); equal up to the order of the float
    # additions in the splat's border overlaps
    b = bunny_c3_small.border
    full = gpu_c3.render(bunny_c3_small.params(), b)
    acc = np.zeros_like(full)
    for r in range(n):
        share = gpu_c3.render(bunny_c3_small.params(tile_stride=n, tile_offset=r), b)
        assert share[..., 4].sum() > 0
        acc += share
    np.testing.assert_allclose(acc, full, rtol=2e-5, atol=2e-6)


def _long_params(scene):
    # ~4 C3 frames of work at 1280x720 (several wavefront batches)
    return scene.params(tile_w=1280, tile_h=720, spp=1024)


@pytest.fixture(scope="module")
def c3_full():
    return mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 1280, "height": 720, "spp": 4})


def test_cancel_from_a_second_thread_stops_the_render(c3_full):
    g = mtsg.GPUScene(c3_full, 0)
    b = c3_full.border
    p = _long_params(c3_full)
    result = {}

    def work():
        t0 = time.time()
        try:
            g.render(p, b)
            result["rc"] = 0
        except RuntimeError as e:
            result["err"] = str(e)
        result["secs"] = time.time() - t0

    th = threading.Thread(target=work)
    th.start()
    time.sleep(0.15)
    g.cancel()
    th.join(60)
    assert not th.is_alive()
    assert "err" in result and "(-4)" in result["err"] and "cancelled" in result["err"], result
    # the handle stays usable and the flag was consumed
    small = c3_full.params(tile_w=64, tile_h=64, spp=1)
    assert g.render(small, b)[..., 4].sum() > 0
    g.close()


def test_cancel_before_render_applies_to_the_next_render_only(c3_full):
    g = mtsg.GPUScene(c3_full, 0)
    b = c3_full.border
    small = c3_full.params(tile_w=64, tile_h=64, spp=1)
    g.cancel()
    with pytest.raises(RuntimeError, match="cancelled"):
        g.render(small, b)
    assert g.render(small, b)[..., 4].sum() > 0
    g.close()


def test_path_job_cancel(c3_full):
    job = mtsg.PathJob(c3_full, 1)
    p = _long_params(c3_full)
    result = {}

    def work():
        result["rc"], _, result["secs"] = job.render(p, c3_full.border)

    th = threading.Thread(target=work)
    th.start()
    time.sleep(0.15)
    job.cancel()
    th.join(60)
    assert not th.is_alive()
    assert result["rc"] == mtsg.MTSG_ERR_CANCELLED, (result, job.last_error())
    # cancel() while idle has no effect: the next render completes
    job.cancel()
    rc, img, _ = job.render(c3_full.params(tile_w=64, tile_h=64, spp=1), c3_full.border)
    assert rc == 0 and img[..., 4].sum() > 0
    job.close()


def test_path_job_reports_the_failing_gpu(c3_full):
    job = mtsg.PathJob(c3_full, 1)
    rc, _, _ = job.render(c3_full.params(spp=0), c3_full.border)
    assert rc == -1
    assert job.last_error().startswith("GPU 0: spp")
    job.close()


def test_path_job_cancel_racing_the_end_of_a_render(c3_full):
    """cancel() calls that land around the moment a render returns never
    leave a stale flag behind: the job's next render completes (ADVICE r02:
    mtsh_path_job_cancel's check-then-cancel window)."""
    job = mtsg.PathJob(c3_full, 1)
    small = c3_full.params(tile_w=128, tile_h=64, spp=2)
    stop = threading.Event()

    def spam():
        while not stop.is_set():
            job.cancel()
    for _ in range(20):
        th = threading.Thread(target=spam)
        th.start()
        rc, _, _ = job.render(small, c3_full.border)
        stop.set()
        th.join()
        stop.clear()
        assert rc in (0, mtsg.MTSG_ERR_CANCELLED), job.last_error()
        rc, img, _ = job.render(small, c3_full.border)
        assert rc == 0, job.last_error()
        assert img[..., 4].sum() > 0
    job.close()


def test_plugin_flow_with_overriding_defines():
    """INTEGRATION.md's plugin: Mitsuba parsed the scene with -D width/height/
    spp/maxDepth; the plugin passes the values it holds in memory to
    mtsh_scene_load_overrides in preprocess(), creates the job once, and
    render() goes through mtsh_path_job_render.  The block has the overridden
    size and the image equals the one of the scene loaded with the same -D
    map (up to the order of the film's float additions)."""
    from test_plugin_overrides import overrides_for
    xml = os.path.join(SCENES, "bunny15.xml")
    by_defines = mtsg.Scene(xml, {"width": 96, "height": 40, "spp": 3, "maxDepth": 5})
    by_plugin = mtsg.Scene(xml, {}, overrides=overrides_for(96, 40, 3, max_depth=5))
    p = by_plugin.params()
    assert (p.tile_w, p.tile_h, p.spp, p.max_depth) == (96, 40, 3, 5)
    job = mtsg.PathJob(by_plugin, 0)
    rc, img, _ = job.render(p, by_plugin.border)
    assert rc == 0, job.last_error()
    b = by_plugin.border
    assert img.shape == (40 + 2 * b, 96 + 2 * b, 5)
    job.close()
    ref_job = mtsg.PathJob(by_defines, 0)
    rc, ref, _ = ref_job.render(by_defines.params(), by_defines.border)
    ref_job.close()
    assert rc == 0
    # the same samples; the film's float atomics add them in any order
    np.testing.assert_allclose(img, ref, rtol=1e-5, atol=1e-6)


def test_crop_window_through_the_job_equals_the_rectangle(tmp_path):
    """An hdrfilm crop (film.cpp:36-48) rendered through the job (the plugin's
    render()) equals the same rectangle of the uncropped scene on the device,
    and the oracle's crop render."""
    from oracle import pyoracle as O
    from test_crop import cropped_xml
    defs = {"width": 320, "height": 180, "spp": 4}
    cropped = mtsg.Scene(cropped_xml(tmp_path, "bunny15.xml", dict(x=100, y=40, w=72, h=56)), defs)
    full = mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), defs)
    p = cropped.params()
    assert (p.tile_x, p.tile_y, p.tile_w, p.tile_h) == (100, 40, 72, 56)
    job = mtsg.PathJob(cropped, 0)
    rc, img, _ = job.render(p, cropped.border)
    job.close()
    assert rc == 0
    g = mtsg.GPUScene(full, 0)
    rect = g.render(full.params(tile_x=100, tile_y=40, tile_w=72, tile_h=56), full.border)
    g.close()
    np.testing.assert_allclose(img, rect, rtol=1e-5, atol=1e-6)
    ref, _ = O.render(cropped.desc, p, cropped.border, rng=O.RNG_COUNTER)
    b = cropped.border
    d = np.abs(mtsg.develop(img[b:-b, b:-b]) - mtsg.develop(ref[b:-b, b:-b]))
    assert d.mean() < 1e-3 * mtsg.develop(ref[b:-b, b:-b]).mean()


def _tiles_of(p):
    out = set()
    for ty in range((p.tile_h + 15) // 16):
        for tx in range((p.tile_w + 15) // 16):
            out.add((p.tile_x + 16 * tx, p.tile_y + 16 * ty, min(16, p.tile_w - 16 * tx), min(16, p.tile_h - 16 * ty)))
    return out


def test_tile_callbacks_report_every_tile_once(bunny_c3_small):
    """mtsg_set_tile_callback / mtsh_path_job_set_tile_callback: every tile of a
    render is reported once, with its rectangle, after its samples are in the
    block -- with small batches (several per frame, so reports arrive while
    the frame renders) and through the job (the plugin's signalWorkEnd /
    progress hook, renderproc.cpp:144-154)."""
    s = bunny_c3_small
    p = s.params(tile_x=8, tile_y=4, tile_w=300, tile_h=170)
    g = mtsg.GPUScene(s, 0)
    seen = []
    g.set_tile_callback(lambda key, x, y, w, h: seen.append((key, x, y, w, h)))
    g.set_batch_paths(16 * 16 * p.spp * 40)   # 40 tiles per batch
    img = g.render(p, s.border)
    assert img[..., 4].sum() > 0
    assert len(seen) == len({k for k, *_ in seen}) == len(_tiles_of(p))
    assert {r[1:] for r in seen} == _tiles_of(p)
    # a share: only its tiles
    seen.clear()
    q = p.copy()
    q.tile_stride, q.tile_offset = 3, 2
    g.render(q, s.border)
    assert seen and all(k % 3 == 2 for k, *_ in seen)
    g.set_tile_callback(None)
    seen.clear()
    g.render(p, s.border)
    assert not seen
    g.close()
    job = mtsg.PathJob(s, 0)
    got = []
    job.set_tile_callback(lambda gpu, x, y, w, h: got.append((gpu, x, y, w, h)))
    rc, _, _ = job.render(p, s.border)
    job.close()
    assert rc == 0
    assert sorted(r[1:] for r in got) == sorted(_tiles_of(p))
    assert {r[0] for r in got} <= set(range(mtsg.device_lib().mtsg_device_count()))
