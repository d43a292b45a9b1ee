#!/usr/bin/env python3
"""Host time of the eager cfg3 train step by function (GPU box): the functions on the path to the raster forward are
wrapped with perf_counter accumulators, 30 steps after 10 warm ones, each step started after a synchronisation (the
bench's first timed step); prints the host time at which each C entry point is first called in the step, and mean us
per step, inclusive, of the wrapped functions in call order."""
import collections
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gstex_amd import _lib, activations, fused, loss, model, ops  # noqa: E402
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
wrap(tr, "zero_grad", "trainer.zero_grad")
wrap(tr, "render", "trainer.render")
wrap(fused, "train_render", "fused.train_render")
wrap(tr, "_run_pending_texture", "trainer._run_pending_texture")
wrap(tr, "_poll_pairs", "trainer._poll_pairs")
wrap(tr.pairs, "scan", "PairCapacity.scan")
wrap(model, "activate", "activate()")
wrap(model, "sh_rest", "sh_rest()")
wrap(ops, "preprocess")
wrap(ops, "bin_capped")
wrap(ops, "texture_gaussians")
wrap(ops, "_launch")
wrap(activations, "call", "activations.call")
wrap(loss, "call", "loss.call")
first_fwd = []
first_call = collections.defaultdict(list)  # C entry point -> host time of its first call in the step
inner_ops, inner_lib = ops.call, _lib.call


n = 30
for _ in range(n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    seen = {}

    def marker(inner):
        def m(name, *a):
            seen.setdefault(name, time.perf_counter() - t0)
            return inner(name, *a)
        return m
    ops.call, _lib.call = marker(inner_ops), marker(inner_lib)
    step()
    ops.call, _lib.call = inner_ops, inner_lib
    for name, t in seen.items():
        first_call[name].append(t)
torch.cuda.synchronize()
fwd = [v for k, v in first_call.items() if k.startswith("gstex_raster_fwd")][0]
print(f"host time to the raster forward launch: median {1e6 * sorted(fwd)[n // 2]:.0f} us")
print("first call of each entry point in the step (median us after the step starts):")
for name, v in sorted(first_call.items(), key=lambda kv: sorted(kv[1])[len(kv[1]) // 2]):
    print(f"  {name:36s} {1e6 * sorted(v)[len(v) // 2]:8.0f}")
for label in order:
    print(f"  {label:32s} {1e6 * acc[label] / n:8.1f} us/step  ({calls[label] / n:.1f} calls)")
