"""The C-ABI library exists, loads, and exports every symbol include/*.h
declares (no compute calls: this runs without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import REPO


def declared(header):
    text = open(os.path.join(REPO, "include", header)).read()
    return sorted(set(re.findall(r"\b(mtsg_[a-z_]+|mtsh_[a-z_]+)\s*\(", text)))


def exported(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", lib]).decode()
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


def test_device_library_exports_abi():
    lib = os.path.join(REPO, "my-mitsuba_amd", "libmtsg.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-C", REPO, "device"])
    names = declared("mtsg.h")
    assert "mtsg_render" in names and "mtsg_scene_create" in names
    missing = [n for n in names if n not in exported(lib)]
    assert not missing, missing
    ctypes.CDLL(lib)   # loads without a GPU present


def test_host_library_exports_api():
    lib = os.path.join(REPO, "my-mitsuba_amd", "libmtsg_host.so")
    names = declared("mtsh.h")
    missing = [n for n in names if n not in exported(lib)]
    assert not missing, missing


def test_python_binding_lists_match_headers():
    import mtsg
    assert sorted(mtsg.DEVICE_SYMBOLS) == declared("mtsg.h")
    assert sorted(mtsg.HOST_SYMBOLS) == declared("mtsh.h")


def test_path_library_exports_api():
    lib = os.path.join(REPO, "my-mitsuba_amd", "libmtsg_path.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-C", REPO, "all"])
    names = declared("mtsg_path.h")
    import mtsg
    assert names == sorted(mtsg.PATH_SYMBOLS)
    missing = [n for n in names if n not in exported(lib)]
    assert not missing, missing
