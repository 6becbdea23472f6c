#!/usr/bin/env python3
"""Extract the Sobol' generator matrices of the reference's sobol sampler
(src/samplers/sobolseq.cpp: Joe & Kuo's new-joe-kuo-6.21201 direction
numbers, 1024 dimensions x 52 columns, as Gruenschloss's tables) as DATA into
a little-endian binary file the host library embeds:

  'SOBT' | u32 dims | u32 columns | u32 vdc rows | u32 vdc_inv rows | 12 zero bytes |
  u32 matrices32[dims * columns] | u64 vdc_sobol_matrices[rows][columns] |
  u64 vdc_sobol_matrices_inv[inv rows][columns]

(row m-1 of vdc_sobol_matrices is used by look_up at resolution 2^m: 25 rows,
the inverse table has 26)

(rows of the vdc tables shorter than `columns` are zero-filled, as C
aggregate initialisation does).  tests/test_sobol.py pins the extracted
columns against the direction numbers regenerated from Joe & Kuo's published
primitive polynomials and initial values.

usage: python tools/extract_sobol_tables.py /root/reference/src/samplers/sobolseq.cpp my-mitsuba_amd/data/sobol_tables.bin
"""
import re
import struct
import sys

src = open(sys.argv[1]).read()


def block(name):
    i = src.index(name)
    j = src.index("};", i)
    return src[src.index("{", i) + 1:j]


m32 = [int(v, 16) for v in re.findall(r"0x([0-9a-fA-F]+)U\b", block("Matrices::matrices32["))]


def rows(name):
    body = block(name)
    out = []
    for r in re.findall(r"\{([^{}]*)\}", body):
        vals = [int(v, 16) for v in re.findall(r"0x([0-9a-fA-F]+)ULL", r)]
        out.append(vals + [0] * (52 - len(vals)))
    return out


vdc = rows("Matrices::vdc_sobol_matrices[]")
inv = rows("Matrices::vdc_sobol_matrices_inv[]")
assert len(m32) == 1024 * 52, len(m32)
with open(sys.argv[2], "wb") as f:
    f.write(b"SOBT" + struct.pack("<IIII", 1024, 52, len(vdc), len(inv)) + bytes(12))   # 32-B header: u64 tables 8-B aligned
    f.write(struct.pack(f"<{len(m32)}I", *m32))
    for t in (vdc, inv):
        for r in t:
            f.write(struct.pack("<52Q", *r))
print(f"matrices32: {len(m32)} words, vdc rows: {len(vdc)}, inverse rows: {len(inv)}")
