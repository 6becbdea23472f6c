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
    r = subprocess.run([os.path.join(REPO, "tools", "check_glibc_mathf"), "97", "sinf", "cosf", "sincosf.s", "sincosf.c",
                        "tanf", "expf", "logf", "atanf", "acosf", "atan2f"], capture_output=True, text=True,
                       timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.strip().splitlines()
    names = {line.split()[0] for line in lines}
    assert {"sinf", "cosf", "sincosf.s", "sincosf.c", "tanf", "expf", "logf", "atanf", "acosf", "atan2f"} <= names
    for line in lines:
        assert re.search(r" 0 differ$", line), line


def test_powf_log2_table_is_its_definition():
    """e_powf_log2_data.c: the 16 subintervals' 1/c are logf's, and log2(c)
    is -log2(1/c) correctly rounded to double."""
    src = open(HDR).read()
    invc = re.findall(r"(-?0x[0-9a-f.]+p[-+]?\d+)", src[src.index("kLogfInvc[16]"):src.index("kLogfLogc[16]")])
    logc = re.findall(r"(-?0x[0-9a-f.]+p[-+]?\d+)", src[src.index("kPowfLogc[16]"):src.index("powf_checkint")])
    assert len(invc) == 16 and len(logc) == 16
    getcontext().prec = 60
    ln2 = Decimal(2).ln()
    for a, b in zip(invc, logc):
        assert float(-(Decimal(float.fromhex(a)).ln() / ln2)) == float.fromhex(b), (a, b)


def test_glibc_powf_over_the_kernels_exponents():
    r = subprocess.run([os.path.join(REPO, "tools", "check_glibc_mathf"), "97", "powf"], capture_output=True, text=True,
                       timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) >= 40 and any("random argument pairs" in line for line in lines)
    for line in lines:
        assert re.search(r" 0 differ$", line), line
