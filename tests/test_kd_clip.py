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
