#!/usr/bin/env python3
"""Per-launch kernel durations of the last frame of a rocprofv3 kernel trace,
in dispatch order (one frame = from a k_camera dispatch to the next), so two
builds that render the same rays (e.g. the MTSG_SHUFFLE coherence variants)
can be compared launch by launch.

  tools/launch_times.py LABEL=DIR/kt_kernel_trace.csv [LABEL=...] > profiles/r06_ray_order.txt"""
import csv
import sys


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return n[:i]
    return n


def last_frame(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [(short(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows
            if not r["Kernel_Name"].startswith("__amd")]
    starts = [i for i, (n, _) in enumerate(rows) if n == "k_camera"]
    return rows[starts[-1]:] if starts else rows


def main():
    runs = []
    for arg in sys.argv[1:]:
        label, path = arg.split("=", 1)
        runs.append((label, last_frame(path)))
    print("# per-launch durations (us) of the last frame, dispatch order; k_reset / copies omitted")
    kinds = ("k_trace_s", "k_shade", "k_finish", "k_tie", "k_camera", "k_splat")
    for label, rows in runs:
        print(f"## {label}")
        tot = {}
        for n, us in rows:
            base = n.split("<")[0]
            if base == "k_reset":
                continue
            tot[base] = tot.get(base, 0.0) + us
            print(f"  {n:45s} {us:10.1f}")
        print("  totals (ms): " + ", ".join(f"{k} {tot[k] / 1e3:.2f}" for k in kinds if k in tot))
    if len(runs) >= 2:
        print("## k_trace_s launch by launch (us)")
        traces = [[us for n, us in rows if n.startswith("k_trace_s")] for _, rows in runs]
        print("  launch " + " ".join(f"{label:>12s}" for label, _ in runs))
        for i in range(max(len(t) for t in traces)):
            print(f"  {i:6d} " + " ".join(f"{t[i]:12.1f}" if i < len(t) else " " * 12 for t in traces))


if __name__ == "__main__":
    main()
