"""The device's float transcendentals (my-mitsuba_amd/csrc/glibc_mathf.h)
against this machine's glibc, the library Mitsuba and the oracle call
(include/mitsuba/core/math.h:175-221; src/emitters/envmap.cpp:386-387,606-607;
src/bsdfs/microfacet.h:573-697).  The header is compiled for the host by
tools/check_glibc_mathf and compared bit for bit over every 97th float bit
pattern (44M arguments per function; the full 2^32 sweep is the tool's
stride-1 run, profiles/r04_glibc_mathf_exhaustive.txt); the same header on the
GPU: tools/math_probe (tests/test_gpu_math.py).  The exp2f table is
recomputed from its definition, round(2^(i/32)) - (i << 47)."""
import os
import re
import struct
import subprocess
from decimal import Decimal, getcontext

from conftest import REPO

HDR = os.path.join(REPO, "my-mitsuba_amd", "csrc", "glibc_mathf.h")


def test_exp2f_table_is_its_definition():
    src = open(HDR).read()
    body = src[src.index("constexpr uint64_t kExp2fTab"):src.index("float expf(float x)")]
    tab = [int(v, 16) for v in re.findall(r"(0x[0-9a-f]+)ull", body)]
    assert len(tab) == 32
    getcontext().prec = 60
    ln2 = Decimal(2).ln()
    for i, t in enumerate(tab):
        u = struct.unpack("<Q", struct.pack("<d", float((ln2 * i / 32).exp())))[0]
        assert (u - (i << 47)) & (2**64 - 1) == t, i


def test_glibc_mathf_matches_libm_bit_for_bit():
    r = subprocess.run([os.path.join(REPO, "tools", "check_glibc_mathf"), "97"], capture_output=True, text=True,
                       timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.strip().splitlines()
    names = {line.split()[0] for line in lines}
    assert {"sinf", "cosf", "sincosf.s", "sincosf.c", "tanf", "expf", "logf", "atanf", "acosf", "atan2f"} <= names
    for line in lines:
        assert re.search(r" 0 differ$", line), line
