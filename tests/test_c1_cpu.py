"""Config C1 (BASELINE.json configs[0]): the Cornell box with the `path`
integrator and the independent sampler at 256x256x16 spp, default maxDepth
(-1, unbounded), rendered on the CPU only -- the reference's own plumbing:
XML load through the host scene library, then the CPU restatement of
SamplingIntegrator::render with SFMT-19937 per-block samplers and 32x32
spiral blocks (integrator.cpp:99-197, imageproc.cpp:28-78,
independent.cpp:51-116), against the counter-mode RNG the GPU uses.  Both
are unbiased estimators of the same image: their means agree within the
noise of 16M-sample frame means, pixel by pixel they differ like two seeds."""
import os

import numpy as np

from conftest import SCENES


def test_c1_cornell_box_cpu():
    import mtsg
    from oracle import pyoracle as O
    scene = mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {})
    p = scene.params()
    assert (p.tile_w, p.tile_h, p.spp, p.max_depth, p.rr_depth) == (256, 256, 16, -1, 5)
    b = scene.border
    sfmt, st = O.render(scene.desc, p, b, rng=O.RNG_SFMT)
    assert st.samples == 256 * 256 * 16
    imgs = []
    for seed in (0, 1):
        p.seed = seed
        imgs.append(O.render(scene.desc, p, b, rng=O.RNG_COUNTER)[0])
    dev = [mtsg.develop(i[b:-b, b:-b]).astype(np.float64) for i in (sfmt, *imgs)]
    for d in dev:
        assert np.isfinite(d).all() and (d >= 0).all()
    # every pixel got its filter weight (gaussian rfilter, no holes)
    for i in (sfmt, *imgs):
        assert (i[b:-b, b:-b, 4] > 0).all()
    m_sfmt, m0, m1 = (d.mean((0, 1)) for d in dev)
    assert (m_sfmt > 0.01).all()
    # frame means: relative spread of two counter seeds sets the noise scale
    noise = np.abs(m0 - m1) + 2e-3 * m0
    assert (np.abs(m_sfmt - m0) < 5 * noise).all(), (m_sfmt, m0, m1)
    l1_cross = np.abs(dev[0] - dev[1]).mean()
    l1_seeds = np.abs(dev[1] - dev[2]).mean()
    assert 0.8 * l1_seeds < l1_cross < 1.25 * l1_seeds, (l1_cross, l1_seeds)
