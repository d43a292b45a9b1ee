#!/usr/bin/env python3
"""Host-side cost of one cfg3 train step (GPU box): cProfile of a few steps of the bench's step() with the device
running ahead of nothing (torch.cuda.synchronize() before each profiled step, like the bench's first timed step), and
the host time from the step's start to each C-ABI launch of the first render (where the device waits for the host)."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gstex_amd import _lib, ops  # noqa: E402
from gstex_amd.model import GStexTrainer  # noqa: E402
from gstex_amd.scene import make_scene, sphere_view  # noqa: E402


def main():
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
    # launch timestamps of one step, relative to its start
    marks = []
    real_call = _lib.call

    def traced(name, *args):
        marks.append((name, time.perf_counter()))
        return real_call(name, *args)

    from gstex_amd import activations, loss

    mods = [m for m in (ops, activations, loss) if hasattr(m, "call")]
    _lib.call = traced
    for m in mods:
        m.call = traced
    t0 = time.perf_counter()
    step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    _lib.call = real_call
    for m in mods:
        m.call = real_call
    print(f"host enqueue of one step after a synchronisation: {1e3 * (t1 - t0):.3f} ms")
    for name, t in marks:
        print(f"  +{1e3 * (t - t0):7.3f} ms  {name}")
    pr = cProfile.Profile()
    for _ in range(5):
        torch.cuda.synchronize()
        pr.enable()
        step()
        pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(30)


if __name__ == "__main__":
    main()
