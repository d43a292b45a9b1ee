#!/usr/bin/env python3
"""Print one training step's kernel timeline (start offset, duration, gaps) from a rocprofv3 --kernel-trace CSV:
    python3 tools/step_timeline.py gpurun_out/quick/run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adams = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
s, e = adams[-2] + 1, adams[-1] + 1
t0 = int(rows[s]["Start_Timestamp"])
prev_end = t0
busy = 0
for r in rows[s:e]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = st - prev_end
    busy += en - st
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:64]
    print(f"{(st - t0) / 1000:8.1f} {(en - st) / 1000:7.1f} gap {gap / 1000:6.1f}  {name}")
    prev_end = en
span = int(rows[e - 1]["End_Timestamp"]) - t0
print(f"step span {span / 1000:.1f} us, kernels busy {busy / 1000:.1f} us, idle {(span - busy) / 1000:.1f} us")
