"""Share balancing on the host (mtsg.balance_order / balance_cuts, the same
order and update as libmtsg_path's job, my-mitsuba_amd/host/path_integrator.cc):
the golden-ratio key order cuts into runs spread over the whole frame, and the
cut follows measured rates while keeping every tile dealt exactly once."""
import numpy as np

import mtsg

TILES = 80 * 45   # the C3 frame's 16x16 tiles


def test_order_is_a_permutation_whose_runs_cover_the_frame():
    o = mtsg.balance_order(TILES)
    assert sorted(o.tolist()) == list(range(TILES))
    # a run of 1/8 of the keys touches every tile row and at least 3/4 of the
    # tile columns (the stride deal touches them all)
    for r in range(8):
        run = o[r * TILES // 8:(r + 1) * TILES // 8]
        ty = run // 80
        assert len(set(ty.tolist())) == 45
        tx = (run % 80 + ty) % 80
        assert len(set(tx.tolist())) >= 60


def test_cuts_follow_rates_and_keep_the_total():
    counts = np.array([450] * 8)
    same = mtsg.balance_cuts(counts, [0.0225] * 8)
    assert same.tolist() == counts.tolist()
    t = np.array([22.3, 22.4, 22.4, 23.0, 23.2, 22.5, 22.5, 22.3]) * 1e-3
    new = mtsg.balance_cuts(counts, t)
    assert new.sum() == TILES
    assert new[4] < 450 and new[0] > new[4] and new[3] < 450
    # the predicted times (rates unchanged) are closer together
    pred = new * (t / counts)
    assert pred.max() - pred.min() < t.max() - t.min()


def test_cuts_keep_one_tile_and_hand_out_the_remainder():
    new = mtsg.balance_cuts([5, 5, 5], [100.0, 1e-3, 1e-3], damping=1.0)
    assert new.sum() == 15 and new.min() >= 1
    new = mtsg.balance_cuts([1, 1, 1, 1], [1.0, 2.0, 3.0, 4.0])
    assert new.tolist() == [1, 1, 1, 1]


def test_put_tile_windows_with_keys_matches_the_stride_form():
    rng = np.random.default_rng(0)
    tile_w, tile_h, b = 100, 70, 2
    n_tiles = 7 * 5
    win = rng.random((n_tiles, 20, 20, 5)).astype(np.float32)
    a = mtsg.put_tile_windows(np.zeros((74, 104, 5), np.float32), win[:12], tile_w, tile_h, b, 3, 1)
    keys = 1 + 3 * np.arange(12)
    k = mtsg.put_tile_windows(np.zeros((74, 104, 5), np.float32), win[:12], tile_w, tile_h, b, 1, 0, keys=keys)
    np.testing.assert_array_equal(a, k)
    # a permuted list with its windows permuted alike gives the same block
    perm = rng.permutation(12)
    k2 = mtsg.put_tile_windows(np.zeros((74, 104, 5), np.float32), win[:12][perm], tile_w, tile_h, b, 1, 0,
                               keys=keys[perm])
    np.testing.assert_allclose(k2, k, rtol=1e-6)


def test_balance_cuts_needs_a_tile_per_share():
    """fewer tiles than shares used to loop forever; bench.py then
    keeps the stride deal instead of balancing."""
    import pytest
    with pytest.raises(ValueError):
        mtsg.balance_cuts([1, 1, 0, 0], [0.1, 0.1, 0.1, 0.1])
