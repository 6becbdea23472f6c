"""Config C4 at its size: the 1280x720 C3 frame (1,041,765 triangles) tiled
over 8 ranks.  Each rank's share is the tiles of deal key k % 8 == r; a rank
returns one ImageBlock per tile (mtsg_render_device_tiles, Mitsuba's per-block
ImageBlocks of BlockedRenderProcess) and the host puts them into the frame
(ImageBlock::put, src/librender/imageblock.h:103-107; the merge of
src/librender/imageproc.cpp:28-78).  The eight shares are rendered one after
the other on this GPU, through the device library and through the integrator's
job API (mtsh_path_job_render), summed, and compared with the whole frame;
the whole frame is compared with the CPU oracle.  (bench.py's N-rank path:
tests/test_gpu_00_bench_ranks.py.)"""
import os

import numpy as np
import pytest

import mtsg
from conftest import SCENES
from oracle import pyoracle as O

pytestmark = pytest.mark.gpu

RANKS = 8


@pytest.fixture(scope="module")
def c3():
    return mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 1280, "height": 720, "spp": 2})


@pytest.fixture(scope="module")
def whole(c3):
    g = mtsg.GPUScene(c3, 0)
    try:
        yield g.render(c3.params(), c3.border)
    finally:
        g.close()


def test_c4_eight_shares_as_tile_imageblocks(c3, whole):
    p = c3.params()
    b = c3.border
    g = mtsg.GPUScene(c3, 0)
    frame = np.zeros_like(whole)
    tiles = 0
    try:
        for r in range(RANKS):
            q = p.copy()
            q.tile_stride, q.tile_offset = RANKS, r
            n, w = g.tile_windows(q)
            assert w == 16 + 2 * b
            nbytes = n * w * w * 5 * 4
            buf = g.alloc(nbytes)
            try:
                g.render_device_tiles(q, buf)
                win = g.download(buf, (n, w, w, 5))
            finally:
                g.free(buf)
            assert (win[..., 4].reshape(n, -1).sum(1) > 0).all()   # every tile of the share has samples
            mtsg.put_tile_windows(frame, win, p.tile_w, p.tile_h, b, RANKS, r)
            tiles += n
    finally:
        g.close()
    assert tiles == 80 * 45
    # the same samples (global RNG keys); the film's float additions differ in order
    np.testing.assert_allclose(frame, whole, rtol=2e-5, atol=2e-6)


def test_c4_eight_shares_through_the_path_job(c3, whole):
    p = c3.params()
    job = mtsg.PathJob(c3, 1)
    acc = np.zeros_like(whole)
    try:
        for r in range(RANKS):
            q = p.copy()
            q.tile_stride, q.tile_offset = RANKS, r
            rc, img, _ = job.render(q, c3.border)
            assert rc == 0, job.last_error()
            acc += img
    finally:
        job.close()
    np.testing.assert_allclose(acc, whole, rtol=2e-5, atol=2e-6)


def test_c4_whole_frame_matches_the_oracle(c3, whole):
    p = c3.params()
    b = c3.border
    ref, _ = O.render(c3.desc, p, b, rng=O.RNG_COUNTER)
    g, c = mtsg.develop(whole[b:-b, b:-b]), mtsg.develop(ref[b:-b, b:-b])
    d = np.abs(g - c)
    mean = float(c.mean())
    assert mean > 0
    assert d.mean() < 1e-3 * mean, (d.mean(), mean)
    px = d.mean(-1)
    print(f"C4 frame 1280x720x2spp: L1 {d.mean():.3e} (mean {mean:.4f}), p99 {np.percentile(px, 99):.2e}, "
          f"max {px.max():.2e}, frac>1e-3 {(px > 1e-3).mean():.2e}")
    # the north star's per-pixel bar, pixel for pixel: with the device's
    # float transcendentals restated from glibc (glibc_mathf.h) every sample
    # of this frame follows the oracle's path
    assert px.max() < 1e-3, px.max()


def test_c4_uneven_tile_lists_sum_to_the_whole_frame(c3, whole):
    """Balanced shares (mtsg_set_tile_list): eight uneven runs of the
    golden-ratio key order, as bench.py's balancing cuts them, rendered as tile
    ImageBlocks in list order, sum to the whole frame."""
    p = c3.params()
    b = c3.border
    order = mtsg.balance_order(80 * 45)
    counts = np.array([300, 520, 410, 480, 455, 470, 505, 460])
    assert counts.sum() == 80 * 45
    g = mtsg.GPUScene(c3, 0)
    frame = np.zeros_like(whole)
    try:
        for r in range(RANKS):
            lo = int(counts[:r].sum())
            keys = np.sort(order[lo:lo + counts[r]])
            g.set_tile_list(keys)
            n, w = g.tile_windows(p)
            assert n == counts[r]
            buf = g.alloc(n * w * w * 5 * 4)
            try:
                g.render_device_tiles(p, buf)
                win = g.download(buf, (n, w, w, 5))
            finally:
                g.free(buf)
            assert (win[..., 4].reshape(n, -1).sum(1) > 0).all()
            mtsg.put_tile_windows(frame, win, p.tile_w, p.tile_h, b, 1, 0, keys=keys)
        # a list in another order renders the same block
        g.set_tile_list(order[:64][::-1])
        q = p.copy()
        blk_list = g.render(q, b)
        g.set_tile_list(np.sort(order[:64]))
        blk_sorted = g.render(q, b)
        np.testing.assert_allclose(blk_list, blk_sorted, rtol=2e-5, atol=2e-6)   # (splat atomics: any order)
        # errors: a repeated key at the call, a key outside the rectangle at the render
        with pytest.raises(RuntimeError, match="distinct"):
            g.set_tile_list([3, 5, 3])
        g.set_tile_list([80 * 45])
        with pytest.raises(RuntimeError, match="outside the rectangle"):
            g.render(q, b)
        g.set_tile_list(None)
        np.testing.assert_allclose(g.render(q, b), whole, rtol=2e-5, atol=2e-6)
    finally:
        g.close()
    np.testing.assert_allclose(frame, whole, rtol=2e-5, atol=2e-6)


def test_path_job_rebalances_between_renders(c3, whole):
    """mtsh_path_job re-cuts its GPUs' shares from the last render's rates; on
    one GPU the only share is the whole tile set, and a second render of the
    same set keeps it (the image does not depend on the cut)."""
    p = c3.params()
    job = mtsg.PathJob(c3, 1)
    try:
        for _ in range(2):
            rc, img, secs = job.render(p, c3.border)
            assert rc == 0, job.last_error()
            tiles, s = job.shares()
            assert tiles.tolist() == [80 * 45] and s[0] > 0
            np.testing.assert_allclose(img, whole, rtol=2e-5, atol=2e-6)
        job.set_balance(False)
        rc, img, _ = job.render(p, c3.border)
        assert rc == 0
        np.testing.assert_allclose(img, whole, rtol=2e-5, atol=2e-6)
    finally:
        job.close()
