#!/usr/bin/env python3
"""Per-launch HBM traffic of the dominant kernel from rocprofv3 --pmc passes.

Reads <dir>/fetch_counter_collection.csv (FETCH_SIZE) and
<dir>/write_counter_collection.csv (WRITE_SIZE), and <dir>/stats_kernel_stats.csv.
Corrections per MI355X_MICROARCH.md "HBM": FETCH_SIZE is KB of 64-B-tallied
128-B requests on gfx950 -> x2; WRITE_SIZE is exact for 16-B/lane stores.
Both count Infinity-Cache hits (memory-side requests), so this is an upper
bound on DRAM bytes.  Only the timed kernel variant is used (the bench's
instrumented COUNT pass runs a separately named instantiation)."""
import csv
import json
import os
import sys

KERNEL = "k_trace_s<false, 16, false>"


def launches(path, counter):
    out = []
    for row in csv.DictReader(open(path)):
        if KERNEL in row["Kernel_Name"] and row["Counter_Name"] == counter:
            out.append(float(row["Counter_Value"]))
    return out


d = sys.argv[1]
f = launches(os.path.join(d, "fetch_counter_collection.csv"), "FETCH_SIZE")
w = launches(os.path.join(d, "write_counter_collection.csv"), "WRITE_SIZE")
stats = {}
p = os.path.join(d, "stats_kernel_stats.csv")
if os.path.exists(p):
    for row in csv.DictReader(open(p)):
        if KERNEL in row["Name"]:
            stats = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]), "total_ns": float(row["TotalDurationNs"])}
fetch_b = 2 * 1024 * sum(f) / max(1, len(f))     # KB -> B, gfx950 x2
write_b = 1024 * sum(w) / max(1, len(w))
print(json.dumps({
    "kernel": KERNEL, "workload": "bunny15", "launches_fetch_pass": len(f), "launches_write_pass": len(w),
    "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
    "traffic_bytes_per_launch": fetch_b + write_b, "rocprof_stats": stats,
    "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE; counts Infinity-Cache hits (memory-side requests)",
}, indent=1))
