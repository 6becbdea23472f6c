"""Statistical parity of the RNG substitution (SURVEY §8c "statistical
parity"): the product keys its random numbers by (pixel, sample, dimension)
 where the reference draws from per-core SFMT-19937 streams
(src/samplers/independent.cpp:51-116, src/libcore/random.cpp).  Both must be
unbiased estimators of the same image: renders of the CPU restatement in the
two RNG modes agree to within their own sample noise."""
import os

import numpy as np

from conftest import SCENES


def develop(block, b):
    import mtsg
    return mtsg.develop(block[b:-b, b:-b]).astype(np.float64)


def test_counter_rng_matches_sfmt_statistically():
    import mtsg
    from oracle import pyoracle as O
    scene = mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {"width": 48, "height": 48, "spp": 128})
    p = scene.params(max_depth=6)
    b = scene.border
    counter = []
    for seed in range(6):
        p.seed = seed
        img, _ = O.render(scene.desc, p, b, rng=O.RNG_COUNTER)
        counter.append(develop(img, b))
    sfmt_img, st = O.render(scene.desc, p, b, rng=O.RNG_SFMT)
    sfmt = develop(sfmt_img, b)
    assert st.samples == 48 * 48 * 128
    means = np.array([c.mean((0, 1)) for c in counter])          # (seeds, 3)
    mu, sd = means.mean(0), means.std(0, ddof=1)
    z = np.abs(sfmt.mean((0, 1)) - mu) / (sd * np.sqrt(1 + 1 / len(counter)))
    assert np.all(z < 5), (z, mu, sfmt.mean((0, 1)))
    # per-pixel: SFMT-vs-counter differences look like counter-vs-counter noise
    l1_cross = np.abs(sfmt - counter[0]).mean()
    l1_noise = np.mean([np.abs(counter[i] - counter[0]).mean() for i in range(1, len(counter))])
    assert 0.8 * l1_noise < l1_cross < 1.25 * l1_noise, (l1_cross, l1_noise)
