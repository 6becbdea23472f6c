"""The oracle (CPU restatement) pinned against the reference's own
known-answer vectors and invariants."""
import json
import os

import numpy as np

from oracle import pyoracle as O
from conftest import GOLDEN


def test_sfmt_matches_reference_kat():
    # src/tests/test_random.cpp:433-507 -- 192 nextULong() of Random(4321)
    g = json.load(open(os.path.join(GOLDEN, "sfmt_seed4321.json")))
    want = [int(v) for v in g["next_ulong"]]
    assert O.sfmt_sequence(4321, len(want)) == want


def test_sfmt_float_construction():
    # random.cpp:629-639: ((u & 0xFFFFFFFF) >> 9) | 0x3f800000, minus 1
    L = O.lib()
    a = L.oracle_sfmt_new(4321)
    b = L.oracle_sfmt_new(4321)
    for _ in range(100):
        u = L.oracle_sfmt_next_ulong(a)
        f = L.oracle_sfmt_next_float(b)
        bits = ((u & 0xFFFFFFFF) >> 9) | 0x3F800000
        assert np.float32(np.array([bits], np.uint32).view(np.float32)[0] - np.float32(1.0)) == np.float32(f)
    L.oracle_sfmt_free(a)
    L.oracle_sfmt_free(b)


def test_sfmt_clone_is_deterministic_and_distinct():
    # Random(Random*) seeding of per-core sampler clones (random.cpp:528-546)
    L = O.lib()
    p1, p2 = L.oracle_sfmt_new(5489), L.oracle_sfmt_new(5489)
    c1, c2 = L.oracle_sfmt_clone(p1), L.oracle_sfmt_clone(p2)
    s1 = [L.oracle_sfmt_next_ulong(c1) for _ in range(16)]
    s2 = [L.oracle_sfmt_next_ulong(c2) for _ in range(16)]
    assert s1 == s2
    c3 = L.oracle_sfmt_clone(p1)   # second clone from the advanced parent
    assert [L.oracle_sfmt_next_ulong(c3) for _ in range(16)] != s1
    for r in (p1, p2, c1, c2, c3):
        L.oracle_sfmt_free(r)


def test_counter_rng_uniform():
    L = O.lib()
    u = np.array([L.oracle_counter_float(0, i, d) for i in range(2000) for d in range(4)], np.float64)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.01
    # different seeds give different streams
    assert L.oracle_counter_float(0, 7, 3) != L.oracle_counter_float(1, 7, 3)
