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
    d, key = sys.argv[1], json.loads(sys.argv[2])
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
        if f and w:
            fb = 2 * 1024 * sum(f) / len(f)
            wb = 1024 * sum(w) / len(w)
            k.update(fetch_bytes_per_launch=fb, write_bytes_per_launch=wb, traffic_bytes_per_launch=fb + wb,
                     traffic_bytes_per_step=fb * len(f) + wb * len(w))
        if h + m > 0:
            k.update(tcc_hit_rate=round(h / (h + m), 4), tcc_launches=len(tcc[name].get("TCC_HIT_sum", [])))
        if name in stats:
            k["rocprof_stats"] = stats[name]
        kernels[name] = k
    print(json.dumps({"key": key, "kernels": kernels,
                      "note": "traffic = FETCH_SIZE x2 (gfx950) + WRITE_SIZE per launch, memory-side requests "
                              "(Infinity-Cache hits included); tcc_hit_rate = TCC_HIT_sum / (HIT + MISS)"}, indent=1))


if __name__ == "__main__":
    main()
