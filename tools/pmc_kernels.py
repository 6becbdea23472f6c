#!/usr/bin/env python3
"""Per-kernel memory traffic and L2 hit rate of one bench configuration from
rocprofv3 passes (each counter group in its own run, as MI355X_MICROARCH.md
prescribes), keyed by the configuration so that bench.py can only ever pick
up counters of the kernel and configuration it ran.

  tools/pmc_kernels.py DIR KEY_JSON > profiles/rNN_pmc_<tag>.json

DIR holds <pass>_counter_collection.csv for the passes fetch (FETCH_SIZE),
write (WRITE_SIZE) and tcc (TCC_HIT_sum, TCC_MISS_sum), and
stats_kernel_stats.csv.  KEY_JSON is bench.py's pmc_key() of the profiled
command (workload, instancing, kd_build, width, height, spp, share).
Corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE counts KB of 64-B-tallied
128-B requests on gfx950 -> x2; WRITE_SIZE is exact for 16-B/lane stores.
Both count Infinity-Cache hits (memory-side requests), so traffic is an
upper bound on DRAM bytes.  The instrumented COUNT instantiations
(k_trace_s<true, ...>) are listed under their own names and never confused
with the timed ones."""
import csv
import json
import os
import sys
from collections import defaultdict


def kernel_name(full):
    """rocprofv3's demangled name without return type, namespace and
    arguments: 'void (anonymous namespace)::k_trace_s<false, 16, false>(mtsg::DevScene, ...)'
    -> 'k_trace_s<false, 16, false>'."""
    n = full.strip()
    if n.startswith("void "):
        n = n[5:]
    n = n.replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return n[:i]
    return n


def per_kernel(path, counters):
    out = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return out
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] in counters:
            out[kernel_name(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return out


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("key")
    ap.add_argument("--frames-stats", type=int, default=0, help="frames the stats pass rendered (bench.py --pmc-pass)")
    ap.add_argument("--frames-pass", type=int, default=0, help="frames each counter pass rendered")
    ap.add_argument("--fetch-factor", type=float, default=2.0,
                    help="FETCH_SIZE correction of the streaming kernels (MI355X_MICROARCH.md: x2 on gfx950)")
    ap.add_argument("--fetch-factor-trace", type=float, default=None,
                    help="correction for the traversal kernels' gathers (profiles/r06_fetch_calibration.txt)")
    a = ap.parse_args()
    d, key = a.dir, json.loads(a.key)
    fetch = per_kernel(os.path.join(d, "fetch_counter_collection.csv"), {"FETCH_SIZE"})
    write = per_kernel(os.path.join(d, "write_counter_collection.csv"), {"WRITE_SIZE"})
    tcc = per_kernel(os.path.join(d, "tcc_counter_collection.csv"), {"TCC_HIT_sum", "TCC_MISS_sum"})
    stats = {}
    p = os.path.join(d, "stats_kernel_stats.csv")
    if os.path.exists(p):
        for row in csv.DictReader(open(p)):
            stats[kernel_name(row["Name"])] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                                               "total_ns": float(row["TotalDurationNs"])}
    kernels = {}
    for name in sorted(set(fetch) | set(write) | set(tcc)):
        f = fetch[name].get("FETCH_SIZE", [])
        w = write[name].get("WRITE_SIZE", [])
        h, m = sum(tcc[name].get("TCC_HIT_sum", [])), sum(tcc[name].get("TCC_MISS_sum", []))
        k = {"launches_fetch_pass": len(f), "launches_write_pass": len(w)}
        trace = name.startswith("k_trace_s") or name.startswith("k_tie") or name.startswith("k_finish")
        factor = a.fetch_factor_trace if (trace and a.fetch_factor_trace is not None) else a.fetch_factor
        if f and w:
            fb = factor * 1024 * sum(f) / len(f)
            wb = 1024 * sum(w) / len(w)
            k.update(fetch_factor=factor, fetch_bytes_per_launch=fb, write_bytes_per_launch=wb,
                     traffic_bytes_per_launch=fb + wb, traffic_bytes_per_pass=fb * len(f) + wb * len(w))
            if a.frames_pass > 0:
                k.update(launches_per_frame=len(f) / a.frames_pass,
                         traffic_bytes_per_frame=(fb * len(f) + wb * len(w)) / a.frames_pass)
        if h + m > 0:
            k.update(tcc_hit_rate=round(h / (h + m), 4), tcc_launches=len(tcc[name].get("TCC_HIT_sum", [])))
        if name in stats:
            k["rocprof_stats"] = stats[name]
        kernels[name] = k
    out = {"key": key, "kernels": kernels}
    if a.frames_pass > 0:
        out.update(frames_fetch_pass=a.frames_pass, frames_stats_pass=a.frames_stats)
        for k in kernels.values():
            if "rocprof_stats" in k and "launches_per_frame" in k:
                k["rocprof_ms_per_frame"] = k["rocprof_stats"]["avg_ns"] * k["launches_per_frame"] / 1e6
    print(json.dumps({**out,
                      "note": "traffic = FETCH_SIZE x fetch_factor (per kernel: x2 for gfx950's streaming reads, "
                              "the calibrated gather factor for the traversal, profiles/r06_fetch_calibration.txt) "
                              "+ WRITE_SIZE per launch, memory-side requests (Infinity-Cache hits included); "
                              "tcc_hit_rate = TCC_HIT_sum / (HIT + MISS); *_per_frame: the pass rendered "
                              "frames_fetch_pass frames (bench.py --pmc-pass)"}, indent=1))


if __name__ == "__main__":
    main()
