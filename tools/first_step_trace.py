#!/usr/bin/env python3
"""The first timed step against a steady step, from a rocprofv3 --kernel-trace CSV of
`bench.py --no-sub --no-cpu-baseline --warmup W`:  python3 tools/first_step_trace.py run_kernel_trace.csv W
A step runs from one activate_fwd kernel to the next (the geometry restore and the previous step's deferred texel
Adam sit just before it); the first timed step is the W-th (0-based; the first warmup step sizes the pair capacity).
Prints the idle time before it, then its kernels (offset, duration beside the median over the timed steps' second
half, idle gap before each)."""
import csv
import statistics as st
import sys


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:44]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
S = [int(r["Start_Timestamp"]) for r in rows]
E = [int(r["End_Timestamp"]) for r in rows]
N = [short(r["Kernel_Name"]) for r in rows]
W = int(sys.argv[2]) if len(sys.argv) > 2 else 5
act = [i for i, n in enumerate(N) if "activate_fwd" in n or "train_splat" in n]
steps = list(zip(act[:-1], act[1:]))
spans = [(S[b] - S[a]) / 1e3 for a, b in steps]
first = W
steady = list(range(W + 10, min(W + 20, len(steps))))
cut = steps[first][0]
k0 = cut - 1
while k0 > 0 and "adam" not in N[k0]:
    k0 -= 1
k0 -= 1  # the last warmup step's geometry Adam: the device's last work before the synchronisation
idle_before = sum(max(0, S[i] - E[i - 1]) for i in range(k0 + 1, cut + 1)) / 1e3
print(f"idle between the last warmup step's Adam and the first timed step's first own kernel: {idle_before:.1f} us")
print(f"first step span {spans[first]:.1f} us, steady median {st.median(spans[k] for k in steady):.1f} us")
a, b = steps[first]
t0 = S[cut]
med = {}
for k in steady:
    sa, sb = steps[k]
    for j, i in enumerate(range(sa, sb)):
        med.setdefault(j, []).append((E[i] - S[i]) / 1e3)
prev = S[a]
idle = 0.0
for j, i in enumerate(range(a, b)):
    gap = max(0, S[i] - prev)
    idle += gap
    m = st.median(med[j]) if j in med else float("nan")
    print(f"  +{(S[i] - t0) / 1e3:8.1f} dur {(E[i] - S[i]) / 1e3:7.1f} (steady {m:7.1f}) gap {gap / 1e3:6.1f}  {N[i]}")
    prev = max(prev, E[i])
busy = sum(E[i] - S[i] for i in range(a, b)) / 1e3
sb_ = [sum(E[i] - S[i] for i in range(*steps[k])) / 1e3 for k in steady]
print(f"first step: busy {busy:.1f} us, idle {idle / 1e3:.1f} us; steady busy median "
      f"{st.median(sb_):.1f} us")
