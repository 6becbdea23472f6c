"""Shared fixtures.  `-m gpu` tests need a gfx950 device and the in-tree
libmtsg.so; everything else runs on the CPU (oracle, host loader, ABI)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "my-mitsuba_amd"))
sys.path.insert(0, REPO)

SCENES = os.path.join(REPO, "scenes")
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libmtsg.so")


def _ensure_built():
    import subprocess
    need = [os.path.join(REPO, p) for p in ("my-mitsuba_amd/libmtsg_host.so", "oracle/liboracle.so",
                                             "oracle/liboracle_fast.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.check_call(["make", "-C", REPO, "-j4", "host", "oracle"])
    if not os.path.exists(os.path.join(REPO, "scenes", "sky512.pfm")):
        subprocess.check_call(["make", "-C", REPO, "scenes/sky512.pfm"])


_ensure_built()


@pytest.fixture(scope="session")
def cbox_small():
    import mtsg
    return mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {"width": 64, "height": 48, "spp": 8})


@pytest.fixture(scope="session")
def bunny_small():
    import mtsg
    return mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 160, "height": 90, "spp": 4})
