"""The reference's Sutherland-Hodgman known-answer test
(src/tests/test_kd.cpp:34-84, TestKDTree::test01_sutherlandHodgman) against
the triangle clipping that the host kd build's perfect splits use
(Triangle::getClippedAABB; my-mitsuba_amd/host/build.cpp clipTriangle,
through mtsh_clip_triangle)."""
import numpy as np

import mtsg

UNIT_TRIANGLE = np.array([0, 0, 0, 1, 0, 0, 1, 1, 0], np.float32)


def clip(box_min, box_max):
    box = np.array(list(box_min) + list(box_max), np.float32)
    out = np.zeros(6, np.float32)
    ok = mtsg.host_lib().mtsh_clip_triangle(UNIT_TRIANGLE.ctypes.data, box.ctypes.data, out.ctypes.data)
    return bool(ok), out[:3], out[3:]


def test_split_in_half():
    ok, mn, mx = clip((0, .5, -1), (1, 1, 1))
    assert ok
    np.testing.assert_array_equal(mn, [.5, .5, 0])
    np.testing.assert_array_equal(mx, [1, 1, 0])


def test_clipped_away():
    ok, _, _ = clip((2, 2, 2), (3, 3, 3))
    assert not ok


def test_box_contains_triangle():
    ok, mn, mx = clip((-1, -1, -1), (1, 1, 1))
    assert ok
    np.testing.assert_array_equal(mn, [0, 0, 0])
    np.testing.assert_array_equal(mx, [1, 1, 0])


def test_flat_cell_keeps_the_triangle():
    ok, mn, mx = clip((-100, -100, 0), (100, 100, 0))
    assert ok
    np.testing.assert_array_equal(mn, [0, 0, 0])
    np.testing.assert_array_equal(mx, [1, 1, 0])


def test_touching_box_gives_a_point():
    ok, mn, mx = clip((0, 1, 0), (1, 2, 0))
    assert ok
    np.testing.assert_array_equal(mn, [1, 1, 0])
    np.testing.assert_array_equal(mx, [1, 1, 0])


def clip_double(tri, lo, hi):
    """Sutherland-Hodgman in double precision (triangle.cpp:70-116), the
    clipped polygon's exact bounds; None when fewer than 3 vertices remain
    before a clip stage."""
    poly = [np.array(v, np.float64) for v in tri]
    for axis in range(3):
        for plane, keep in ((lo[axis], lambda x, p: x >= p), (hi[axis], lambda x, p: x <= p)):
            if len(poly) < 3:
                return None
            out = []
            for i, cur in enumerate(poly):
                nxt = poly[(i + 1) % len(poly)]
                ci, ni = keep(cur[axis], plane), keep(nxt[axis], plane)
                if ci:
                    out.append(cur)
                if ci != ni:
                    t = (plane - cur[axis]) / (nxt[axis] - cur[axis])
                    p = cur + (nxt - cur) * t
                    p[axis] = plane
                    out.append(p)
            poly = out
    if not poly:
        return None
    return np.min(poly, 0), np.max(poly, 0)


def test_clipped_bounds_round_outwards():
    """math::castflt_down / castflt_up (triangle.cpp:134-141): the float box
    encloses the double-precision clipped polygon, within one ulp, so a split
    plane never lands inside a triangle's true extent on the wrong side."""
    rng = np.random.default_rng(7)
    checked = outward = 0
    for _ in range(2000):
        tri = rng.uniform(-1, 1, (3, 3)).astype(np.float32)
        c = rng.uniform(-0.5, 0.5, 3).astype(np.float32)
        h = rng.uniform(0.05, 0.8, 3).astype(np.float32)
        lo, hi = (c - h).astype(np.float32), (c + h).astype(np.float32)
        want = clip_double(tri.astype(np.float64), lo.astype(np.float64), hi.astype(np.float64))
        box = np.concatenate([lo, hi]).astype(np.float32)
        out = np.zeros(6, np.float32)
        ok = mtsg.host_lib().mtsh_clip_triangle(np.ascontiguousarray(tri.ravel()).ctypes.data, box.ctypes.data,
                                                out.ctypes.data)
        assert bool(ok) == (want is not None)
        if want is None:
            continue
        wmn, wmx = np.maximum(want[0], lo), np.minimum(want[1], hi)
        mn, mx = out[:3].astype(np.float64), out[3:].astype(np.float64)
        assert (mn <= wmn).all() and (mx >= wmx).all()
        assert (np.nextafter(out[:3], np.float32(np.inf)) >= wmn.astype(np.float32)).all()
        assert (np.nextafter(out[3:], np.float32(-np.inf)) <= wmx.astype(np.float32)).all()
        checked += 1
        outward += int((mn < wmn).any() or (mx > wmx).any())
    assert checked > 500 and outward > 100
