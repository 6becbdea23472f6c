#!/usr/bin/env python3
"""FETCH_SIZE against known bytes for the access shapes of tools/fetch_calib
(the stream the guide calibrates, and the traversal's gathers).

  tools/fetch_calib_summary.py DIR/fetch_counter_collection.csv RUN.log > profiles/r06_fetch_calibration.txt

For each kernel launch: FETCH_SIZE (KB x 1024) / the bytes the lanes asked
for, / the distinct 128-B lines, / the distinct 64-B sectors.  A shape whose
FETCH_SIZE equals its sectors x 64 B is tallied per 64-B request; one whose
second half-line load adds nothing (g16x2 = g16) fills whole lines."""
import csv
import re
import sys
from collections import defaultdict


def main():
    csv_path, log_path = sys.argv[1], sys.argv[2]
    fetch = defaultdict(list)
    for row in csv.DictReader(open(csv_path)):
        if row["Counter_Name"] == "FETCH_SIZE":
            name = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            fetch[name].append(float(row["Counter_Value"]) * 1024.0)
    known = []
    for line in open(log_path):
        m = re.match(r"(\S+) rep (\d): ([\d.]+) ms, (\d+) bytes requested, (\d+) 128-B lines, (\d+) 64-B sectors", line)
        if m:
            known.append((m.group(1), int(m.group(2)), float(m.group(3)), float(m.group(4)), float(m.group(5)),
                          float(m.group(6))))
    # rocprof lists k_g48 for both offsets: the launch order interleaves them
    seen = defaultdict(int)
    print("# FETCH_SIZE calibration (tools/fetch_calib.hip; rocprofv3 --pmc FETCH_SIZE), one MI355X")
    print(f"{'kernel':12s} {'rep':>3s} {'ms':>8s} {'FETCH_SIZE B':>14s} {'/requested':>10s} {'/lines*128':>10s} "
          f"{'/sectors*64':>11s} {'B/access':>9s}")
    rows = {}
    for name, rep, ms, req, lines, sectors in known:
        kname = name.split("@")[0]
        i = seen[kname]
        seen[kname] += 1
        if i >= len(fetch.get(kname, [])):
            continue
        fb = fetch[kname][i]
        n = 1 << 24
        rows[(name, rep)] = fb
        print(f"{name:12s} {rep:3d} {ms:8.3f} {fb:14.0f} {fb / req:10.3f} {fb / (lines * 128):10.3f} "
              f"{fb / (sectors * 64):11.3f} {fb / n:9.1f}")
    def r(name):
        v = [rows[k] for k in rows if k[0] == name]
        return sum(v) / len(v) if v else float("nan")
    g16, g16x2, g48a, g48b, st = r("k_g16"), r("k_g16x2"), r("k_g48@0"), r("k_g48@48"), r("k_stream16")
    n = 1 << 24
    print()
    print(f"stream16: FETCH_SIZE / bytes = {st / (16.0 * n):.3f} (the guide: 0.5, x2)")
    print(f"g16x2 / g16 = {g16x2 / g16:.3f}; g48@48 / g48@0 = {g48b / g48a:.3f} "
          "(2: each 64-B sector is its own request; 1: whole 128-B lines are filled)")
    print(f"gathers: FETCH_SIZE per touched 64-B sector = {g16 / n:.1f} B (g16), {g16x2 / (2 * n):.1f} B (g16x2), "
          f"{g48a / n:.1f} B (g48@0), {g48b / (2 * n):.1f} B (g48@48)")


if __name__ == "__main__":
    main()
