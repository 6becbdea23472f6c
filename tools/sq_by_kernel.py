#!/usr/bin/env python3
"""SQ counters per kernel instantiation from rocprofv3 --pmc passes (one
counter set per pass, counter_collection.csv each), with the wave-time
fractions that tell issue-bound from latency-bound kernels:
  issue = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES   (a wave issuing)
  wait  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES     (a wave waiting on an
          instruction's operands: memory / LDS latency)
  valu_per_wave = SQ_INSTS_VALU / SQ_WAVES
  tools/sq_by_kernel.py DIR/p1_counter_collection.csv DIR/p2_counter_collection.csv ..."""
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_kernels import kernel_name  # noqa: E402


def main():
    agg = defaultdict(lambda: defaultdict(float))
    for path in sys.argv[1:]:
        for row in csv.DictReader(open(path)):
            agg[kernel_name(row["Kernel_Name"])][row["Counter_Name"]] += float(row["Counter_Value"])
    for k in sorted(agg):
        c = agg[k]
        if not k.startswith(("k_shade", "k_trace", "k_finish", "k_camera", "k_splat")):
            continue
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        line = [f"{k}"]
        if wc:
            line.append(f"issue {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}")
            line.append(f"wait_inst {c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}")
            line.append(f"wait_any {c.get('SQ_WAIT_ANY', 0) / wc:.3f}")
            line.append(f"valu_active {c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}")
        if c.get("SQ_WAVES"):
            line.append(f"valu/wave {c.get('SQ_INSTS_VALU', 0) / c['SQ_WAVES']:.0f}")
            for n in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
                if n in c:
                    line.append(f"{n[9:].lower()}/wave {c[n] / c['SQ_WAVES']:.0f}")
        if c.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in c:
            line.append(f"lds_conflict/inst {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_INSTS_LDS']:.2f}")
        print("  ".join(line))
        print("    " + ", ".join(f"{n} {v:.4g}" for n, v in sorted(c.items())))


if __name__ == "__main__":
    main()
