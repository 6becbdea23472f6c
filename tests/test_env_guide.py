"""The device's envmap importance sampling searches its row / column CDFs
from guide tables (my-mitsuba_amd/csrc/envmap.h env_sample_reuse_guided,
DESIGN §3): for every draw it must return the index, and the remapped sample,
of the full std::lower_bound search that restates sampleReuse
(src/emitters/envmap.cpp:628-633).  tools/check_env_guide compiles both
functions for the host and compares them on each scene's own CDFs, at random
draws and at every guide bucket's edges."""
import os
import subprocess

import pytest

from conftest import REPO, SCENES


@pytest.mark.parametrize("scene", ["env_glass.xml"])
def test_guided_cdf_search_equals_lower_bound(scene):
    r = subprocess.run([os.path.join(REPO, "tools", "check_env_guide"), os.path.join(SCENES, scene), "500"],
                       capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 differ" in r.stdout
