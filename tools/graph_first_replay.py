#!/usr/bin/env python3
"""First vs later replays of the cfg3 step graphs (gstex_amd.graphs.StepGraphs): each replay isolated between two
synchronisations and timed with events, poses 0..7 three times over.  GSTEX_GRAPH_UPLOAD=none|capture|current picks
where hipGraphUpload runs after instantiation."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gstex_amd.graphs import StepGraphs, _UPLOAD  # noqa: E402
from gstex_amd.model import GStexTrainer  # noqa: E402
from gstex_amd.scene import make_scene, sphere_view  # noqa: E402

dev = torch.device("cuda", 0)
scene = make_scene(200_000, 1e7, seed=42)
views = [sphere_view(i, 800, 800, n_views=8).to(dev) for i in range(8)]
tr = GStexTrainer(scene, dev, start_step=3000, defer_texture=True)
g = torch.Generator().manual_seed(1000)
gts = [torch.rand((800, 800, 3), generator=g).to(dev) for _ in range(8)]


def body(k):
    tr.zero_grad()
    tr.forward_backward(views[k], gts[k])
    tr.optimizer_step()


body(0)
body(1)
graphs = StepGraphs(tr, body, 8)
graphs.capture()
if os.environ.get("BUSY_FIRST"):  # the device kept busy after the capture before the first replays (clock ramp?)
    for k in range(6):
        body(k % 8)
    graphs.capture()  # (an eager step in between: re-captured; the capture itself idles the device again)
    x = torch.empty((1 << 28,), device=dev)
    for _ in range(200):
        x.mul_(1.0001)  # ~0.3 s of streaming work right before the replays
rows = []
same = os.environ.get("ROUND0_SAME")  # round 0 replays pose 0 eight times: a per-graph first-launch cost or a ramp?
for rnd in range(3):
    t, h = [], []
    for k in range(8):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        t0 = time.perf_counter()
        graphs.replay(0 if (same and rnd == 0) else k)
        h.append(round(1e3 * (time.perf_counter() - t0), 3))
        b.record()
        torch.cuda.synchronize()
        t.append(round(a.elapsed_time(b), 3))
    rows.append(t)
    print(f"upload={_UPLOAD} round {rnd}: {t} host ms {h}", flush=True)
for k in range(2):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    body(k)
    b.record()
    torch.cuda.synchronize()
    print(f"eager after a sync, pose {k}: {a.elapsed_time(b):.3f} ms")
graphs.close()
