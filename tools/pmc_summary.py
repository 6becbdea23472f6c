#!/usr/bin/env python3
"""Aggregate rocprofv3 counter_collection CSVs per kernel family.
usage: pmc_summary.py file1_counter_collection.csv [...]"""
import csv
import re
import sys
from collections import defaultdict


def family(name):
    if "k_trace" in name:
        return "trace"
    for k in ("k_shade", "k_splat", "k_camera", "k_reset"):
        if k in name:
            return k[2:]
    return "other"


agg = defaultdict(lambda: defaultdict(float))
dur = defaultdict(dict)
for path in sys.argv[1:]:
    for row in csv.DictReader(open(path)):
        f = family(row["Kernel_Name"])
        agg[f][row["Counter_Name"]] += float(row["Counter_Value"])
        dur[f][(path, row["Dispatch_Id"])] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
for f in sorted(agg):
    ms = sum(dur[f].values()) / 1e6
    print(f"{f}: {len(dur[f])} dispatches, {ms:.2f} ms (sum over passes)")
    for k, v in sorted(agg[f].items()):
        print(f"    {k:40s} {v:.4g}")
