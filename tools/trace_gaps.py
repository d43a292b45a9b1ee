#!/usr/bin/env python3
"""Per-step kernel busy time and inter-kernel gaps from rocprofv3 --kernel-trace CSVs (eager vs graph steps):
    python3 tools/trace_gaps.py A_kernel_trace.csv [B_kernel_trace.csv ...]
Steps are delimited by the raster forward's starts; for each file: the median step span, kernel busy time and idle
time over the last half of the steps, and the median gap before each kernel of the step (the largest ones)."""
import csv
import statistics as st
import sys


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]


def analyse(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    fwd = [i for i, r in enumerate(rows) if "raster_fwd_kernel" in r["Kernel_Name"]]
    steps = []
    for a, b in zip(fwd[:-1], fwd[1:]):
        seg = rows[a:b]
        t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
        busy, gaps, prev = 0, [], int(seg[0]["Start_Timestamp"])
        for r in seg:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            busy += e - s
            gaps.append((short(r["Kernel_Name"]), max(0, s - prev)))
            prev = max(prev, e)
        steps.append((t1 - t0, busy, gaps))
    tail = steps[len(steps) // 2:]
    span = st.median(s[0] for s in tail) / 1e3
    busy = st.median(s[1] for s in tail) / 1e3
    print(f"{path}: {len(steps)} steps; last {len(tail)}: span {span:.1f} us, kernels {busy:.1f} us, "
          f"idle {span - busy:.1f} us, {len(tail[0][2])} kernels per step")
    n = min(len(s[2]) for s in tail)
    med = [(tail[0][2][k][0], st.median(s[2][k][1] for s in tail) / 1e3) for k in range(n)]
    for name, g in sorted(med, key=lambda x: -x[1])[:12]:
        print(f"    gap {g:6.1f} us before {name}")


for p in sys.argv[1:]:
    analyse(p)
