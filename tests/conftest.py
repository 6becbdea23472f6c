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
    """Every library the tests load must match its sources: `make -q` checks
    the in-tree .so files against csrc/, host/ and oracle/ (a no-op when they
    are current) and anything stale is rebuilt here, loudly, before any test
    runs -- a prebuilt library that no longer matches the sources is never
    tested silently."""
    import subprocess
    targets = ["host", "device", "oracle", "my-mitsuba_amd/libmtsg_path.so", "scenes/sky512.pfm", "tools/check_glibc_mathf"]
    if subprocess.call(["make", "-C", REPO, "-q"] + targets, stdout=subprocess.DEVNULL) != 0:
        print(f"conftest: rebuilding stale native libraries ({' '.join(targets)})", flush=True)
        subprocess.check_call(["make", "-C", REPO, "-j8"] + targets)


_ensure_built()


@pytest.fixture(scope="session")
def cbox_small():
    import mtsg
    return mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {"width": 64, "height": 48, "spp": 8})


@pytest.fixture(scope="session")
def bunny_small():
    import mtsg
    return mtsg.Scene(os.path.join(SCENES, "bunny15.xml"), {"width": 160, "height": 90, "spp": 4})
