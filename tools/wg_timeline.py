#!/usr/bin/env python3
"""Summarise a GSTEX_STATS=3 per-wave timeline dump of the raster backward (tools/raster_loop.py with
GSTEX_WG_DUMP=<file.npy>): kernel span, wave-duration percentiles, occupancy over time, the longest waves."""
import sys

import numpy as np

a = np.load(sys.argv[1]).astype(np.int64)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
a = a[:n]
a = a[a[:, 0] > 0]  # units that exited before stamping (empty segments) left zeros
t0, t1, depth, wl = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
base = t0.min()
s, e = (t0 - base) / 100.0, (t1 - base) / 100.0  # s_memrealtime: 100 MHz -> us
dur = e - s
T = e.max()
print(f"span {T:.1f} us, {n} waves; duration p50/p90/p99/max {np.percentile(dur, [50, 90, 99, 100]).round(1)}")
print("running waves at fraction of span:", {f: int((s <= f * T).sum() - (e <= f * T).sum())
                                              for f in (0.1, 0.3, 0.5, 0.7, 0.8, 0.9, 0.95)})
print("start-time percentiles", np.percentile(s, [50, 90, 99, 100]).round(1))
for i in np.argsort(-e)[:8]:
    print(f"  wave {i}: start {s[i]:.1f} end {e[i]:.1f} dur {dur[i]:.1f} depth {depth[i]} wave_last {wl[i]}")
