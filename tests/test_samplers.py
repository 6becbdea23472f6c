"""Samplers: halton, hammersley, ldsampler next to independent.

Pinning:
  * the reference's known-answer tests src/tests/test_samplers.cpp:33-83
    (MATLAB haltonset / Hammersley values; the test samplers are created
    without configure(), i.e. without digit permutations, on a 1x1 film);
  * Faure's permutations (Faure 1992, "Good permutations for extreme
    discrepancy": sigma_5 = 0 3 2 1 4, sigma_7 = 0 2 5 3 1 4 6), the
    default scramble = -1 of PermutationStorage (faure.cpp:33-57);
  * properties: the blocked Halton / Hammersley partition puts sample s of
    pixel (x, y) inside that pixel (halton.cpp:240-293), and the ldsampler's
    scrambled (0,2)-sequence is a (0,2)-net per pixel and dimension.
Random digit permutations (scramble > 0, TEA-seeded) and the ldsampler's
per-pixel scramble/shuffle streams have no reference values here: parity
unpinned beyond the properties above."""
import os

import numpy as np
import pytest

import mtsg
from oracle import pyoracle as O
from conftest import SCENES


def sampler_scene(tmp_path, sampler_xml, width=1, height=1, spp=5):
    """The Cornell box with the given <sampler> element and film size."""
    text = open(os.path.join(SCENES, "cbox.xml")).read()
    i, j = text.index("<sampler"), text.index("</sampler>") + len("</sampler>")
    text = text[:i] + sampler_xml + text[j:]
    path = tmp_path / "scene.xml"
    path.write_text(text)
    return mtsg.Scene(str(path), {"width": width, "height": height, "spp": spp})


def draws(scene, x, y, s, kinds, **over):
    return O.sampler_draws(scene.desc, scene.params(**over), x, y, s, kinds)


HALTON_KAT = np.array([
    0, 0, 0, 0, 0,
    0.500000000000000, 0.333333333333333, 0.200000000000000, 0.142857142857143, 0.090909090909091,
    0.250000000000000, 0.666666666666667, 0.400000000000000, 0.285714285714286, 0.181818181818182,
    0.750000000000000, 0.111111111111111, 0.600000000000000, 0.428571428571429, 0.272727272727273,
    0.125000000000000, 0.444444444444444, 0.800000000000000, 0.571428571428571, 0.363636363636364,
]).reshape(5, 5)


def test_halton_known_answers(tmp_path):
    # test_samplers.cpp:33-55: 5 samples x 5 next1D, tolerance 1e-7
    sc = sampler_scene(tmp_path, '<sampler type="halton"><integer name="scramble" value="0"/>'
                                 '<integer name="sampleCount" value="$spp"/></sampler>')
    for i in range(5):
        np.testing.assert_allclose(draws(sc, 0, 0, i, [1] * 5), HALTON_KAT[i], atol=1e-7, rtol=0)


def test_hammersley_known_answers(tmp_path):
    # test_samplers.cpp:57-80: sampleCount 5, 5 samples x 6 next1D
    sc = sampler_scene(tmp_path, '<sampler type="hammersley"><integer name="scramble" value="0"/>'
                                 '<integer name="sampleCount" value="$spp"/></sampler>', spp=5)
    for i in range(5):
        want = np.concatenate([[i / 5.0], HALTON_KAT[i]])
        np.testing.assert_allclose(draws(sc, 0, 0, i, [1] * 6), want, atol=1e-7, rtol=0)


def test_faure_permutations(tmp_path):
    # scramble -1 (the default): the digit of index s < b in base b is sigma_b(s)
    sc = sampler_scene(tmp_path, '<sampler type="halton"><integer name="sampleCount" value="$spp"/></sampler>', spp=8)
    sigma = {5: [0, 3, 2, 1, 4], 7: [0, 2, 5, 3, 1, 4, 6]}
    for dim, b in ((2, 5), (3, 7)):
        got = [draws(sc, 0, 0, s, [1] * (dim + 1))[dim] for s in range(b)]
        np.testing.assert_allclose(got, np.array(sigma[b]) / b, atol=1e-7, rtol=0)


def test_random_permutations_are_permutations(tmp_path):
    sc = sampler_scene(tmp_path, '<sampler type="halton"><integer name="scramble" value="7"/>'
                                 '<integer name="sampleCount" value="$spp"/></sampler>', spp=16)
    for dim, b in ((0, 2), (1, 3), (2, 5), (4, 11)):
        v = np.array([draws(sc, 0, 0, s, [1] * (dim + 1))[dim] for s in range(b)])
        assert np.all((v >= 0) & (v < 1))
        # v(s) = (sigma(s) + sigma(0) / (b - 1)) / b (the permuted zero digits
        # form a geometric tail, qmc.cpp:99-112): a permutation sigma puts the
        # b values 1/b apart
        np.testing.assert_allclose(np.diff(np.sort(v)), 1.0 / b, atol=1e-6)


@pytest.mark.parametrize("kind", ["halton", "hammersley"])
def test_blocked_partition_places_samples_in_their_pixel(tmp_path, kind):
    # setFilmResolution(crop, blocked = true): the first next2D of sample s of
    # pixel (x, y) is that pixel's jitter in [0, 1)^2 (halton.cpp:365-386)
    sc = sampler_scene(tmp_path, f'<sampler type="{kind}"><integer name="sampleCount" value="$spp"/></sampler>',
                       width=40, height=24, spp=8)
    for y in range(0, 24, 5):
        for x in range(0, 40, 3):
            for s in range(8):
                a, b = draws(sc, x, y, s, [2])
                assert -1e-5 <= a < 1 + 1e-5 and -1e-5 <= b < 1 + 1e-5, (kind, x, y, s, a, b)


def test_ldsampler_rounds_sample_count_and_is_a_02_net(tmp_path):
    sc = sampler_scene(tmp_path, '<sampler type="ldsampler"><integer name="sampleCount" value="12"/>'
                                 '<integer name="dimension" value="3"/></sampler>', width=8, height=8)
    assert sc.info.spp == 16            # ldsampler.cpp:90-94: next power of two
    n = 16
    # 2D requests 0..3 and 1D requests 0..4 interleaved; requests 3+ are past
    # `dimension` and drawn independently (ldsampler.cpp:202-216)
    kinds = [2, 1, 2, 1, 2, 2, 1, 1, 1]
    for (x, y) in ((0, 0), (5, 3)):
        v = np.array([draws(sc, x, y, s, kinds) for s in range(n)])
        assert np.all((v >= 0) & (v < 1))
        two_d = [(0, 1), (3, 4), (6, 7)]          # the low-discrepancy 2D requests
        for i, j in two_d:
            pts = v[:, [i, j]]
            for a in range(5):                     # elementary intervals 2^-a x 2^-(4-a)
                cells = np.floor(pts[:, 0] * 2 ** a).astype(int) * 2 ** (4 - a) + \
                        np.floor(pts[:, 1] * 2 ** (4 - a)).astype(int)
                assert len(set(cells.tolist())) == n, (x, y, i, a)
        for i in (2, 5, 10):                       # the low-discrepancy 1D requests
            assert sorted(np.floor(v[:, i] * n).astype(int).tolist()) == list(range(n))
    # different pixels are scrambled differently
    assert not np.array_equal(draws(sc, 0, 0, 0, kinds), draws(sc, 1, 0, 0, kinds))


def test_halton_dimension_limit(tmp_path):
    # halton.cpp:356-360: requests past the 1024-prime table are an error
    sc = sampler_scene(tmp_path, '<sampler type="halton"><integer name="sampleCount" value="$spp"/></sampler>', spp=4)
    draws(sc, 0, 0, 0, [1] * 1024)
    with pytest.raises(RuntimeError):
        draws(sc, 0, 0, 0, [1] * 1025)


def test_unknown_sampler_is_rejected(tmp_path):
    with pytest.raises(RuntimeError):
        sampler_scene(tmp_path, '<sampler type="stratified"/>')
