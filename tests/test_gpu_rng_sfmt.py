"""The independent-sampler half of the north star on the GPU: the device's
counter-mode random numbers (keyed by pixel, sample and dimension)
against Mitsuba's own generator, the oracle's SFMT-19937 mode with the
reference's default seed 5489 and per-worker clones over spiral blocks
(src/samplers/independent.cpp:51-116, src/libcore/random.cpp:473-533,
renderjob.cpp:57-69).  The two RNGs cannot give the same samples, so the
bar is statistical (SURVEY §8c "statistical parity"), on config C1 (Cornell
box 256x256x16 spp, maxDepth -1):
  * per channel, the SFMT image mean lies within 3 sigma of the GPU's, sigma
    estimated from 16 GPU renders with independent counter seeds;
  * per pixel, GPU-vs-SFMT L1 is SFMT-vs-SFMT noise (the oracle at seed 5489
    against an independent stream, 5490): ratio within [0.8, 1.25].
The SFMT renders run on one oracle thread, so the stream each block gets and
therefore the test's outcome are deterministic."""
import os

import numpy as np
import pytest

import mtsg
from conftest import SCENES
from oracle import pyoracle as O

pytestmark = pytest.mark.gpu


def test_gpu_counter_rng_matches_mitsuba_sfmt_on_c1():
    scene = mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {})
    p, b = scene.params(), scene.border
    assert (p.tile_w, p.tile_h, p.spp, p.max_depth) == (256, 256, 16, -1)

    def dev(img):
        return mtsg.develop(img[b:-b, b:-b]).astype(np.float64)

    g = mtsg.GPUScene(scene, 0)
    gpu = []
    try:
        for seed in range(16):
            q = p.copy()
            q.seed = seed
            gpu.append(dev(g.render(q, b)))
    finally:
        g.close()
    sfmt = []
    for seed in (0, 1):   # 5489 (Mitsuba's default) and 5490
        q = p.copy()
        q.seed = seed
        img, st = O.render(scene.desc, q, b, rng=O.RNG_SFMT, threads=1)
        assert st.samples == 256 * 256 * 16
        sfmt.append(dev(img))
    means = np.array([x.mean((0, 1)) for x in gpu])
    mu, sd = means.mean(0), means.std(0, ddof=1)
    z = np.abs(sfmt[0].mean((0, 1)) - mu) / (sd * np.sqrt(1 + 1 / len(gpu)))
    l1_cross = np.abs(gpu[0] - sfmt[0]).mean()
    l1_sfmt = np.abs(sfmt[1] - sfmt[0]).mean()
    l1_gpu = np.abs(gpu[1] - gpu[0]).mean()
    print(f"C1: GPU mean {mu}, sigma {sd}, SFMT mean {sfmt[0].mean((0, 1))}, z {z}; per-pixel L1 GPU-vs-SFMT "
          f"{l1_cross:.5f}, SFMT-vs-SFMT {l1_sfmt:.5f}, GPU-vs-GPU {l1_gpu:.5f}")
    assert np.all(z < 3), z
    assert 0.8 * l1_sfmt < l1_cross < 1.25 * l1_sfmt, (l1_cross, l1_sfmt)
    assert 0.8 * l1_gpu < l1_cross < 1.25 * l1_gpu, (l1_cross, l1_gpu)
