#!/usr/bin/env python3
"""L2 (TCC) hit rate of the traversal kernel from a rocprofv3 --pmc pass of
TCC_HIT_sum and TCC_MISS_sum: hit / (hit + miss), summed over the timed
kernel's launches (MI355X_MICROARCH.md "L2 (per XCD)")."""
import csv
import json
import os
import sys

KERNEL = "k_trace_s<false, 16, false>"

d = sys.argv[1]
hit = miss = 0.0
n = 0
for row in csv.DictReader(open(os.path.join(d, "tcc_counter_collection.csv"))):
    if KERNEL not in row["Kernel_Name"]:
        continue
    if row["Counter_Name"] == "TCC_HIT_sum":
        hit += float(row["Counter_Value"])
        n += 1
    elif row["Counter_Name"] == "TCC_MISS_sum":
        miss += float(row["Counter_Value"])
print(json.dumps({"kernel": KERNEL, "workload": sys.argv[2] if len(sys.argv) > 2 else "bunny15", "launches": n,
                  "tcc_hit": hit, "tcc_miss": miss, "tcc_hit_rate": round(hit / max(1.0, hit + miss), 4),
                  "note": "TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum) over the launches of one bench step"}, indent=1))
