#!/usr/bin/env python3
"""Raster-only driver for profiling: cfg3 (200k splats, 1e7 texels, 800x800), texture_gaussians
forward + backward repeated --iters times on one view (used under rocprofv3 for profiles/)."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gstex_amd import ops  # noqa: E402
from gstex_amd.scene import make_scene, sphere_view  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--n-splats", type=int, default=200_000)
    ap.add_argument("--n-texels", type=float, default=1e7)
    ap.add_argument("--size", type=int, default=800)
    ap.add_argument("--opacity", type=float, default=0.1)
    ap.add_argument("--no-geometry", action="store_true", help="geometry_outputs=False (training path)")
    ap.add_argument("--photometric", action="store_true",
                    help="upstream gradients on img/alpha/tex only (the training step's case)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sc = make_scene(args.n_splats, args.n_texels, seed=42, opacity=args.opacity if args.opacity > 0 else None)
    v = sphere_view(0, args.size, args.size).to(dev)
    means, scales, quats, opac = [t.to(dev) for t in sc.activated()]
    uv0, umap, vmap = [t.to(dev) for t in sc.uv_mapping()]
    rgbs = torch.rand((sc.n, 3), device=dev)
    tex = sc.texture.to(dev)
    dims = sc.texture_dims.to(dev)
    for t in (means, scales, quats, opac, rgbs, tex):
        t.requires_grad_(True)
    intr = (v.fx, v.fy, v.cx, v.cy)
    g = torch.Generator(device="cpu").manual_seed(0)
    ups = [torch.randn(s, generator=g).to(dev) * 1e-3 for s in
           [(args.size, args.size, 3), (args.size, args.size), (args.size, args.size), (args.size, args.size),
            (args.size, args.size, 3), (args.size, args.size, 3)]]

    def run():
        _, depths = ops.project_points(means, v.viewmat, intr)
        c, e = ops.get_aabb_2d(means, scales, 1, quats, v.viewmat, intr)
        nth = ops.get_num_tiles_hit_2d(c, e, args.size, args.size, 16)
        outs = ops.texture_gaussians((sc.n, 1, 3), dims, c, e, depths, nth, rgbs, opac, means, scales, 1, quats,
                                     uv0, umap, vmap, tex, v.viewmat, v.c2w, v.fx, v.fy, v.cx, v.cy, args.size,
                                     args.size, 16, (1 << 9) | (1 << 10), background=None,
                                     geometry_outputs=not args.no_geometry)
        if args.photometric:
            torch.autograd.backward([outs[0], outs[3], outs[4]], [ups[0], ups[3], ups[4]])
        else:
            torch.autograd.backward(list(outs), ups)
        return nth

    nth = run()
    torch.cuda.synchronize()
    ops.set_kernel_timing(True, names={"gstex_bin_sort", "gstex_raster_setup", "gstex_raster_fwd", "gstex_raster_bwd",
                                      "gstex_raster_setup_bwd", "gstex_raster_setup_bwd_aabb"})
    t0 = time.perf_counter()
    for _ in range(args.iters):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.iters
    kt = {k.replace("gstex_", ""): round(sum(v) / len(v), 3) for k, v in ops.kernel_times().items()}
    ops.set_kernel_timing(False)
    from gstex_amd import _lib
    lib = _lib.load()
    if hasattr(lib, "gstex_debug_stats"):  # GSTEX_STATS=1 builds: backward work counters over all launches
        import ctypes
        buf = (ctypes.c_ulonglong * 24)()
        lib.gstex_debug_stats(buf)
        n = args.iters + 1
        names = ["units", "visits", "visits_any", "contrib_lanes", "flush_passes", "tail_lanes", "flushed_entries", "tex_visits",
                 "fwd_candidates", "fwd_cull_pass", "fwd_visits", "fwd_visits_any", "fwd_contrib_lanes",
                 "bwd_alive_lanes", "bwd_visits_le16", "bwd_visits_ge48", "disjoint_runs", "disjoint_runs_le2",
                 "disjoint_runs_le4", "dense_passes", "half_visits_contrib", "merged_passes", "merge_disjoint"]
        if os.environ.get("GSTEX_STATS_PHASES"):  # GSTEX_STATS=2: wave-clock sums per backward phase
            names = ["load+barrier", "place+cull", "visits", "barrier_pre_combine", "combine+flush", "barrier_end",
                     "prologue", "-"]
        print("stats/launch:", {k: round(v / n) for k, v in zip(names, buf)})
    if hasattr(lib, "gstex_debug_wg") and os.environ.get("GSTEX_WG_DUMP"):  # GSTEX_STATS=3: last launch's waves
        import ctypes
        import numpy as np
        buf = (ctypes.c_ulonglong * (65536 * 4))()
        lib.gstex_debug_wg(buf)
        np.save(os.environ["GSTEX_WG_DUMP"], np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4))
    print(f"fwd+bwd+preprocess {dt * 1e3:.3f} ms/iter  visible={int((nth > 0).sum())} isect={int(nth.sum())} "
          f"kernel_ms={kt}")


if __name__ == "__main__":
    main()
