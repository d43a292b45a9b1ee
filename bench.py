#!/usr/bin/env python3
"""GStex train-step benchmark on MI355X (the metric of BASELINE.json):
"train-step ms + rendered Mpix/s, 200k splats / 1e7 texels @ 800x800".

One step = one full GStex training iteration per rank on synthetic random-init data
(gstex_amd.model.GStexTrainer): activations -> project/AABB/tiles -> SH -> texture_gaussians
fwd -> composite -> 0.8 L1 + 0.2 (1-SSIM) -> backward -> [RCCL all-reduce of the flat gradient
buffer when N > 1] -> 7-group Adam.  Every rank renders its own camera (cfg4: one view per GPU).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Rank 0 prints ONE JSON line.  `value` = whole-job rendered+trained Mpix/s = N * H * W / step time.
`roofline` prices the dominant raster kernel with SURVEY §8d's algorithmic bytes; `cpu_baseline`
times the CPU oracle (oracle/, fp32 forward + autograd backward) on a bounded crop of the same view.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PROFILE_TAG = "r01"  # profiles/<tag>_traffic.json: PMC HBM bytes per launch (tools/profile_bench.sh)


def pmc_row(kernel):
    """`kernel`'s row of the committed rocprofv3 PMC summary: HBM bytes per launch (2 x FETCH_SIZE +
    WRITE_SIZE, separate passes, gfx950 FETCH_SIZE halving corrected) and VALU instructions per launch;
    None if not profiled."""
    path = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_traffic.json")
    try:
        rows = json.load(open(path))["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    for r in rows:
        if r["kernel"].startswith(kernel + "_kernel") and r.get("hbm_bytes_per_launch"):
            return r
    return None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--n-splats", type=int, default=200_000)
    p.add_argument("--n-texels", type=float, default=1e7)
    p.add_argument("--height", type=int, default=800)
    p.add_argument("--width", type=int, default=800)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-crop", type=int, default=96, help="side of the crop the CPU oracle renders")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--no-kernel-timing", action="store_true",
                   help="diagnostics only: no HIP events around the raster launches (no roofline figures)")
    return p.parse_args()


def algorithmic_bytes(nth, dims, H, W, C=3):
    """SURVEY §8d per-kernel algorithmic bytes (counted N_v, T_v, I, P)."""
    vis = nth > 0
    Nv = int(vis.sum())
    I = int(nth.long().sum())
    Tv = int((dims[vis, 0].long() * dims[vis, 1].long()).sum())
    P = H * W
    fwd = 116 * Nv + 4 * I + 4 * C * Tv + 4 * (9 + C) * P + 8 * P
    bwd = 172 * Nv + 4 * I + 8 * C * Tv + 8 * P + 4 * (9 + C) * P
    return dict(N_v=Nv, I=I, T_v=Tv, P=P, fwd=fwd, bwd=bwd)


def cpu_baseline(scene, view, crop, threads):
    """Oracle (fp32 forward + autograd backward) on a crop x crop window at the image centre."""
    from oracle import raster as O

    torch.set_num_threads(threads)
    x0 = view.W // 2 - crop // 2
    y0 = view.H // 2 - crop // 2
    cam = O.Camera(view.viewmat, view.fx, view.fy, view.cx - x0, view.cy - y0, crop, crop, 16, view.c2w[:3, 3])
    means, scales, quats, opac = scene.activated()
    centers, extents = O.aabb_2d(means, scales, 1.0, quats, cam)
    _, depths = O.project_points(means, cam)
    uv0, umap, vmap = scene.uv_mapping()
    g = torch.Generator().manual_seed(0)
    rgbs = torch.rand((scene.n, 3), generator=g)
    leaves = dict(rgbs=rgbs, opacities=opac.detach().clone(), means=means.detach().clone(),
                  scales=scales.detach().clone(), quats=quats.detach().clone(), texture=scene.texture.clone())
    for t in leaves.values():
        t.requires_grad_(True)
    inp = O.RasterInputs(scene.texture_dims, centers.detach(), extents, depths, leaves["rgbs"], leaves["opacities"],
                         leaves["means"], leaves["scales"], 1.0, leaves["quats"], uv0, umap, vmap, leaves["texture"],
                         cam)
    t0 = time.perf_counter()
    bins = O.bin_and_sort(inp.centers, inp.extents, inp.depths, crop, crop)
    out = O._render(inp, torch.float32, bins[1], bins[2], None)["out"]
    loss = sum(v.sum() for k, v in out.items() if k in ("img", "tex", "alpha", "depth"))
    loss.backward()
    dt = time.perf_counter() - t0
    return dict(value=round(crop * crop / dt / 1e6, 6), unit="Mpix/s", cores=threads, kind="port",
                sample=f"oracle fp32 fwd+bwd of a {crop}x{crop} centre crop of the same 800x800 view "
                       f"({scene.n} splats, {scene.texture.shape[0]} texels), {dt:.1f} s wall")


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # "nccl" is RCCL on ROCm; GSTEX_DIST_BACKEND=gloo rehearses several ranks on one GPU
        dist.init_process_group(os.environ.get("GSTEX_DIST_BACKEND", "nccl"), init_method="env://")
    dev_idx = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)

    from gstex_amd import ops
    from gstex_amd.dist import GradSync
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    H, W = args.height, args.width
    t_scene = time.perf_counter()
    scene = make_scene(args.n_splats, args.n_texels, seed=args.seed)
    view = sphere_view(rank, H, W, n_views=max(world, 8)).to(dev)
    trainer = GStexTrainer(scene, dev)
    sync = GradSync(trainer, world) if world > 1 else None
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    gt = torch.rand((H, W, 3), generator=g).to(dev)
    setup_s = time.perf_counter() - t_scene

    def step():
        if sync is not None:
            sync.zero()  # one fill of the flat gradient buffer the .grad views live in
        else:
            trainer.zero_grad()
        trainer.forward_backward(view, gt)
        if sync is not None:
            sync.all_reduce()
        trainer.optimizer_step()

    for _ in range(args.warmup):
        step()
    # counted quantities for the roofline (this rank's view, current parameters)
    with torch.no_grad():
        means = trainer.means
        quats = trainer.quats / trainer.quats.norm(dim=-1, keepdim=True)
        s = torch.exp(trainer.scales[:, :-1])
        scales = torch.cat([s, 1e-5 * s.mean(-1, keepdim=True)], -1)
        intr = (view.fx, view.fy, view.cx, view.cy)
        c, e = ops.get_aabb_2d(means, scales, 1, quats, view.viewmat, intr)
        nth = ops.get_num_tiles_hit_2d(c, e, H, W, 16)
        ab = algorithmic_bytes(nth.cpu(), trainer.texture_dims.cpu(), H, W)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ops.set_kernel_timing(not args.no_kernel_timing)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kt = ops.kernel_times()
    ops.set_kernel_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    mpix = world * H * W / (elapsed / args.steps) / 1e6

    avg = {k: sum(v) / len(v) for k, v in kt.items()}
    f_ms = avg.get("gstex_raster_fwd", float("nan"))
    b_ms = avg.get("gstex_raster_bwd", float("nan"))
    dom, dom_ms, dom_bytes = ("raster_bwd", b_ms, ab["bwd"]) if b_ms >= f_ms else ("raster_fwd", f_ms, ab["fwd"])
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    roofline = dict(bound="hbm", kernel=dom, achieved=round(achieved, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(achieved / HBM_PEAK_GBS, 4), traffic=None,
                    traffic_source=f"profiles/{PROFILE_TAG}_traffic.json",
                    bytes_per_launch=dom_bytes, launch_ms=round(dom_ms, 4),
                    fwd_bwd_frac=round((ab["fwd"] + ab["bwd"]) / ((f_ms + b_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))

    prow = pmc_row(dom)
    if prow is not None:
        roofline["traffic"] = int(prow["hbm_bytes_per_launch"])
        if prow.get("valu_insts"):
            # the kernel is VALU-issue/latency bound, not HBM bound: its issue roofline, live time
            roofline["valu_insts_per_launch"] = int(prow["valu_insts"])
            roofline["valu_issue_frac"] = round(prow["valu_insts"] / (dom_ms * 1e-3 * 1024 * 2.4e9 / 2), 4)

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(make_scene(args.n_splats, args.n_texels, seed=args.seed), sphere_view(0, H, W),
                               args.cpu_crop, min(args.cpu_threads, os.cpu_count() or 1))
        except Exception as ex:  # baseline must never kill the GPU result line
            cpu = dict(value=None, unit="Mpix/s", cores=args.cpu_threads, kind="port", sample=f"failed: {ex!r}")
    line = {
        "metric": "train-step ms + rendered Mpix/s, 200k splats/1e7 texels @800x800",
        "value": round(mpix, 4),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seed 42 random-init splats, charted random texels, random target image)",
        "config": {
            "workload": "cfg3 full GStex train step (fwd+loss+bwd+Adam), one 800x800 view per GPU",
            "n_splats": args.n_splats, "n_texels": int(trainer.texture_dc.shape[0]), "H": H, "W": W,
            "views_per_step": world, "parallelism": f"dp{world}",
        },
        "roofline": roofline,
        "cpu_baseline": cpu,
        "kernel_ms": {k.replace("gstex_", ""): round(v, 4) for k, v in avg.items()},
        "counts": {k: ab[k] for k in ("N_v", "I", "T_v", "P")},
        "setup_s": round(setup_s, 1),
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
