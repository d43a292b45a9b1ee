#!/usr/bin/env python3
"""Host time of the eager cfg3 train step by function (GPU box): the functions on the path to the raster forward are
wrapped with perf_counter accumulators, 30 steps after 10 warm ones, each step started after a synchronisation (the
bench's first timed step); prints mean us per step, inclusive, in call order, and the time to the raster forward."""
import collections
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gstex_amd import _lib, activations, loss, model, ops  # noqa: E402
from gstex_amd.model import GStexTrainer  # noqa: E402
from gstex_amd.scene import make_scene, sphere_view  # noqa: E402

acc = collections.defaultdict(float)
calls = collections.Counter()
order = []


def wrap(mod, name, label=None):
    fn = getattr(mod, name)
    label = label or f"{getattr(mod, '__name__', mod)}.{name}"

    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc[label] += time.perf_counter() - t0
            calls[label] += 1
            if label not in order:
                order.append(label)
    setattr(mod, name, w)


dev = torch.device("cuda", 0)
scene = make_scene(200_000, 1e7, seed=42)
views = [sphere_view(i, 800, 800).to(dev) for i in range(8)]
tr = GStexTrainer(scene, dev, start_step=3000, defer_texture=True)
g = torch.Generator().manual_seed(1000)
gts = [torch.rand((800, 800, 3), generator=g).to(dev) for _ in range(8)]
geom0 = tr.geometry_flat.detach().clone()
k = [0]


def step():
    with torch.no_grad():
        tr.geometry_flat.copy_(geom0)
    tr.zero_grad()
    tr.forward_backward(views[k[0] % 8], gts[k[0] % 8])
    tr.optimizer_step()
    k[0] += 1


for _ in range(10):
    step()
torch.cuda.synchronize()
wrap(tr, "render", "trainer.render")
wrap(tr, "_run_pending_texture", "trainer._run_pending_texture")
wrap(tr, "_poll_pairs", "trainer._poll_pairs")
wrap(tr.pairs, "scan", "PairCapacity.scan")
wrap(model, "activate", "activate()")
wrap(model, "sh_rest", "sh_rest()")
wrap(ops, "preprocess")
wrap(ops, "bin_capped")
wrap(ops, "texture_gaussians")
wrap(ops, "_launch")
wrap(_lib, "call", "_lib.call")
wrap(ops, "call", "ops.call")
wrap(activations, "call", "activations.call")
wrap(loss, "call", "loss.call")
first_fwd = []
inner = ops.call


n = 30
for _ in range(n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    seen = [None]

    def marker(name, *a):
        if name.startswith("gstex_raster_fwd") and seen[0] is None:
            seen[0] = time.perf_counter() - t0
        return inner(name, *a)
    ops.call = marker
    step()
    ops.call = inner
    first_fwd.append(seen[0])
torch.cuda.synchronize()
print(f"host time to the raster forward launch: median {1e6 * sorted(first_fwd)[n // 2]:.0f} us")
for label in order:
    print(f"  {label:32s} {1e6 * acc[label] / n:8.1f} us/step  ({calls[label] / n:.1f} calls)")
