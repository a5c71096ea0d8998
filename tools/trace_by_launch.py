#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_trace.csv per (kernel, launch shape).

usage: trace_by_launch.py <kernel_trace.csv> [> by_launch.csv]
Columns: kernel (name without argument list), grid, wg, arch/accum VGPRs,
scratch, LDS, calls, average and minimum duration in ms; sorted by total time.
"""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0]
            key = (name, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]), int(r["VGPR_Count"]),
                   int(r["Accum_VGPR_Count"]), int(r["Scratch_Size"]), int(r["LDS_Block_Size"]))
            rows[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid", "wg", "arch_vgpr", "accum_vgpr", "scratch", "lds", "calls", "avg_ms", "min_ms"])
    for key, d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        w.writerow(list(key) + [len(d), f"{sum(d) / len(d):.4f}", f"{min(d):.4f}"])


if __name__ == "__main__":
    main(sys.argv[1])
