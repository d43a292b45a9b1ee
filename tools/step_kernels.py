#!/usr/bin/env python3
"""One bench step's kernel timeline from a rocprofv3 --kernel-trace CSV (gpurun_out/pt/trace by default):
start offset, duration and grid of every launch between two consecutive Adam launches, then the per-kernel
totals per step over the whole run."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pt/trace/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
t0 = int(rows[a]["End_Timestamp"])
for r in rows[a + 1:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} grid={r['Grid_Size_X']:>9s} {r['Kernel_Name'][:64]}")
print(f"step span {(int(rows[b]['End_Timestamp']) - t0) / 1e3:.1f} us")
