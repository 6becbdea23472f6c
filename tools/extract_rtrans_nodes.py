#!/usr/bin/env python3
"""Golden fixture for roughplastic's rough transmittance (tests/golden/rtrans_nodes.json).

Reads the reference's precomputed RoughTransmittance tables
(/root/reference/data/microfacet/{beckmann,ggx,phong}.dat; format per
src/bsdfs/rtrans.h:88-145: "MTS_TRANSMITTANCE", three uint64 sizes
(eta, alpha, theta), four float32 ranges (etaMin, etaMax, alphaMin, alphaMax),
then for each of 2*etaSamples blocks and each alpha: thetaSamples values of
T followed by one diffuse transmittance) and keeps a small subset of grid
nodes as data: both eta blocks (eta > 1 and, in the second block, 1/eta),
a few eta and alpha nodes, all theta samples.  The node coordinates follow
the tables' 4th-root warping (rtrans.h:177-207).
"""
import json
import os
import struct
import sys

SRC = "/root/reference/data/microfacet"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "rtrans_nodes.json")


def read_table(path):
    b = open(path, "rb").read()
    assert b[:17] == b"MTS_TRANSMITTANCE"
    o = 17
    ne, na, nt = struct.unpack_from("<QQQ", b, o); o += 24
    emin, emax, amin, amax = struct.unpack_from("<4f", b, o); o += 16
    n = (len(b) - o) // 4
    assert n == 2 * ne * na * (nt + 1)
    vals = struct.unpack_from("<%df" % n, b, o)
    return ne, na, nt, (emin, emax, amin, amax), vals


def main():
    out = {"source": "data/microfacet/*.dat of the reference (Mitsuba 0.6); see tools/extract_rtrans_nodes.py",
           "tables": {}}
    for name, dist in (("beckmann", 0), ("ggx", 1), ("phong", 2)):
        ne, na, nt, (emin, emax, amin, amax), vals = read_table(os.path.join(SRC, name + ".dat"))
        nodes = []
        for block in (0, 1):
            for i in (12, 30, 45):
                for j in (10, 22, 35):
                    if j >= na or i >= ne:
                        continue
                    eta = emin + (emax - emin) * (i / (ne - 1)) ** 4
                    alpha = amin + (amax - amin) * (j / (na - 1)) ** 4
                    base = ((block * ne + i) * na + j) * (nt + 1)
                    nodes.append({"eta": eta if block == 0 else 1.0 / eta, "alpha": alpha,
                                  "trans": [round(v, 7) for v in vals[base:base + nt]],
                                  "diffuse": round(vals[base + nt], 7)})
        out["tables"][name] = {"distribution": dist, "eta_samples": ne, "alpha_samples": na,
                               "theta_samples": nt, "ranges": [emin, emax, amin, amax], "nodes": nodes}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", OUT, sum(len(t["nodes"]) for t in out["tables"].values()), "nodes")


if __name__ == "__main__":
    sys.exit(main())
