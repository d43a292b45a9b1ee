#!/usr/bin/env python3
"""GStex train-step benchmark on MI355X (the metric of BASELINE.json):
"train-step ms + rendered Mpix/s, 200k splats / 1e7 texels @ 800x800".

One step = one full GStex training iteration per rank on synthetic random-init data
(gstex_amd.model.GStexTrainer): activations -> project/AABB/tiles -> SH (degree 3) -> texture_gaussians
fwd -> composite -> 0.8 L1 + 0.2 (1-SSIM) -> backward -> [RCCL all-reduce of the flat gradient buffer when
N > 1] -> 7-group Adam.  Rank r renders camera (r + step * N) mod 8 of 8 fixed sphere poses (the reference
draws one random training camera per rank and step, full_images_datamanager.py:320-333).

The workload is stationary: the geometry parameters that decide which (pixel, splat) pairs exist (means,
log-scales, quaternions, opacity logits; 8.8 MB at cfg3) are restored from their initial values before every
step, inside the timed region, so the pair counts and kernel times do not drift as the scene trains and the
result does not depend on --steps / --warmup.  Colours, texels and the Adam moments keep training.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Rank 0 prints ONE JSON line.  `value` = whole-job rendered+trained Mpix/s = N * H * W / (wall time / K).
`roofline` prices the dominant raster kernel with SURVEY §8d's algorithmic bytes; `cpu_baseline` times the CPU
oracle (oracle/, fp32 forward + autograd backward) on a bounded crop of the same view; `sub` holds the other
configs' kernel times (cfg2 raster fwd+bwd, cfg1 forward), the eval render and a rechart.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PROFILE_TAG = "r06d"  # profiles/<tag>_traffic.json: PMC HBM bytes per launch (tools/profile_bench.sh)
N_POSES = 8


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
    p.add_argument("--steps", type=int, default=30)
    # the device clock and caches settle over the first ~10 steps after the scene setup (measured: 3.16, 2.73,
    # 2.59, 2.52, 2.49 ... 2.40 ms at cfg3 with 5 warmup steps): the default warmup covers that ramp
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--n-splats", type=int, default=200_000)
    p.add_argument("--n-texels", type=float, default=1e7)
    p.add_argument("--height", type=int, default=800)
    p.add_argument("--width", type=int, default=800)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-sub", action="store_true", help="skip the cfg1/cfg2/eval/rechart sub-records")
    p.add_argument("--no-defer-texture", action="store_true",
                   help="run the texel Adam update inside optimizer_step instead of deferring it into the next "
                        "step's render (GStexTrainer defer_texture)")
    p.add_argument("--cpu-crop", type=int, default=96, help="side of the crop the CPU oracle renders")
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


def cpu_threads():
    """Host threads the CPU baseline uses: the CPUs this process may run on (sched affinity), capped by
    OMP_NUM_THREADS when the environment sets it (the GPU box does: its per-GPU CPU share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(n, 1)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def oracle_crop(scene, view, crop, bwd=True):
    """Oracle (fp32 forward [+ autograd backward]) on a crop x crop window at the image centre; seconds."""
    from oracle import raster as O

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
    if bwd:
        for t in leaves.values():
            t.requires_grad_(True)
    inp = O.RasterInputs(scene.texture_dims, centers.detach(), extents, depths, leaves["rgbs"], leaves["opacities"],
                         leaves["means"], leaves["scales"], 1.0, leaves["quats"], uv0, umap, vmap, leaves["texture"],
                         cam)
    t0 = time.perf_counter()
    bins = O.bin_and_sort(inp.centers, inp.extents, inp.depths, crop, crop)
    out = O._render(inp, torch.float32, bins[1], bins[2], None)["out"]
    if bwd:
        loss = sum(v.sum() for k, v in out.items() if k in ("img", "tex", "alpha", "depth"))
        loss.backward()
    return time.perf_counter() - t0


def cpu_baseline(scene, view, crop, threads):
    torch.set_num_threads(threads)
    dt = oracle_crop(scene, view, crop)
    return dict(value=round(crop * crop / dt / 1e6, 6), unit="Mpix/s", cores=threads, kind="port",
                cpu_model=cpu_model(), os_cpu_count=os.cpu_count(),
                sample=f"oracle fp32 fwd+bwd of a {crop}x{crop} centre crop of the same 800x800 view "
                       f"({scene.n} splats, {scene.texture.shape[0]} texels), {dt:.1f} s wall, 1 rep")


def _events_ms(pairs):
    return [a.elapsed_time(b) for a, b in pairs]


def raster_only(n_splats, n_texels, H, W, reps, dev, backward=True, seed=42, opacity=0.1, geo=False):
    """Raster-only fwd(+bwd) median over `reps` on one sphere view: preprocessing
    + binning + texture_gaussians forward [+ backward with img/alpha/tex upstream gradients ~ N(0, 1e-3); geo: every
    output (depth, distortion and normal too, cfg5's depth + normal training) produced and differentiated].
    Returns per-kernel medians, the whole call's median and the roofline fraction of fwd+bwd."""
    from gstex_amd import ops
    from gstex_amd.scene import make_scene, sphere_view

    sc = make_scene(n_splats, n_texels, seed=seed, opacity=opacity)
    v = sphere_view(0, H, W).to(dev)
    means, scales, quats, opac = [t.to(dev) for t in sc.activated()]
    uv0, umap, vmap = [t.to(dev) for t in sc.uv_mapping()]
    rgbs = torch.rand((sc.n, 3), device=dev)
    tex = sc.texture.to(dev)
    dims = sc.texture_dims.to(dev)
    leaves = (means, scales, quats, opac, rgbs, tex)
    if backward:
        for t in leaves:
            t.requires_grad_(True)
    g = torch.Generator(device="cpu").manual_seed(0)
    shapes = [(H, W, 3), (H, W), (H, W), (H, W), (H, W, 3), (H, W, 3)] if geo else [(H, W, 3), (H, W), (H, W, 3)]
    ups = [torch.randn(s, generator=g).to(dev) * 1e-3 for s in shapes]
    intr = (v.fx, v.fy, v.cx, v.cy)

    def run():
        _, depths = ops.project_points(means, v.viewmat, intr)
        c, e = ops.get_aabb_2d(means, scales, 1, quats, v.viewmat, intr)
        nth = ops.get_num_tiles_hit_2d(c, e, H, W, 16)
        outs = ops.texture_gaussians((sc.n, 1, 3), dims, c, e, depths, nth, rgbs, opac, means, scales, 1, quats,
                                     uv0, umap, vmap, tex, v.viewmat, v.c2w, v.fx, v.fy, v.cx, v.cy, H, W, 16,
                                     (1 << 9) | (1 << 10), background=None, geometry_outputs=geo or not backward)
        if backward:
            torch.autograd.backward(list(outs) if geo else [outs[0], outs[3], outs[4]], ups)
            for t in leaves:
                t.grad = None
        return nth

    with torch.no_grad() if not backward else torch.enable_grad():
        nth = run()
        torch.cuda.synchronize()
        ops.set_kernel_timing(True)
        whole = []
        for _ in range(reps):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            run()
            b.record()
            whole.append((a, b))
        kt = ops.kernel_times()
        ops.set_kernel_timing(False)
    ab = algorithmic_bytes(nth.cpu(), sc.texture_dims, H, W)
    med = {k.replace("gstex_", ""): round(statistics.median(v_), 4) for k, v_ in kt.items()}
    res = dict(n_splats=n_splats, n_texels=int(tex.shape[0]), H=H, W=W, reps=reps,
               call_ms_median=round(statistics.median(_events_ms(whole)), 4), kernel_ms_median=med,
               counts={k: ab[k] for k in ("N_v", "I", "T_v", "P")})
    f_ms = med.get("raster_fwd")
    b_ms = med.get("raster_bwd")
    if f_ms:
        res["fwd_hbm_frac"] = round(ab["fwd"] / (f_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
    if f_ms and b_ms:
        res["fwd_bwd_hbm_frac"] = round((ab["fwd"] + ab["bwd"]) / ((f_ms + b_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
    return res


def eval_render_ms(trainer, view, reps):
    """The reference's eval render (gstex.py:1165-1203, measure_fps False): three C = 6 raster calls per image
    (main render, test-colour render, settings | 1 << 15 render), no gradient.  Median ms per image."""
    times = []
    with torch.no_grad():
        trainer.eval_render(view)
        torch.cuda.synchronize()
        for _ in range(reps):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            trainer.eval_render(view)
            b.record()
            times.append((a, b))
        torch.cuda.synchronize()
    return statistics.median(_events_ms(times))


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev_idx = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_idx)  # before the process group: its collectives and barrier() use this rank's GPU
    dev = torch.device("cuda", dev_idx)
    if world > 1:
        # "nccl" is RCCL on ROCm (bound to this rank's GPU); GSTEX_DIST_BACKEND=gloo rehearses several ranks on one GPU
        backend = os.environ.get("GSTEX_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, init_method="env://", device_id=dev if backend == "nccl" else None)

    from gstex_amd import _lib, ops
    from gstex_amd.dist import GradSync
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    H, W = args.height, args.width
    t_scene = time.perf_counter()
    scene = make_scene(args.n_splats, args.n_texels, seed=args.seed)
    views = [sphere_view(i, H, W, n_views=N_POSES).to(dev) for i in range(N_POSES)]
    for v in views:  # each view's camera centre, cached with the view (View.campos), made with the views
        v.campos
    # start_step = 3 x sh_degree_interval: SH at its full degree 3 (the regime of 12k of the 15k iterations)
    trainer = GStexTrainer(scene, dev, start_step=3000, defer_texture=not args.no_defer_texture)
    sync = GradSync(trainer, world) if world > 1 else None
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    gts = [torch.rand((H, W, 3), generator=g).to(dev) for _ in range(N_POSES)]
    geom0 = trainer.geometry_flat.detach().clone()  # means / log-scales / quats / opacity logits, one allocation
    setup_s = time.perf_counter() - t_scene
    step_no = [0]

    def body(pose):
        with torch.no_grad():  # stationary workload: same geometry every step (8.8 MB, one copy, timed)
            trainer.geometry_flat.copy_(geom0)
        if sync is not None:
            sync.zero()  # one fill of the flat gradient buffer the .grad views live in
        else:
            trainer.zero_grad()
        trainer.forward_backward(views[pose], gts[pose])
        # N > 1: the collectives inside the step (texel group updated while the head's collective runs)
        trainer.optimizer_step(sync=sync)

    timed = {"gstex_raster_bwd"} if world == 1 else {"gstex_raster_fwd", "gstex_raster_bwd"}

    def step():
        pose = (rank + step_no[0] * world) % N_POSES
        step_no[0] += 1
        body(pose)

    # counted quantities for the roofline (every pose of this rank's cycle; the geometry is stationary), before the
    # warmup: host work between the warmup and the timed steps would idle the device and let its clock drop
    with torch.no_grad():
        quats = trainer.quats / trainer.quats.norm(dim=-1, keepdim=True)
        s = torch.exp(trainer.scales[:, :-1])
        scales = torch.cat([s, 1e-5 * s.mean(-1, keepdim=True)], -1)
        abs_ = []
        for pose in sorted({(rank + k * world) % N_POSES for k in range(args.steps)}):
            v = views[pose]
            c, e = ops.get_aabb_2d(trainer.means, scales, 1, quats, v.viewmat, (v.fx, v.fy, v.cx, v.cy))
            nth = ops.get_num_tiles_hit_2d(c, e, H, W, 16)
            abs_.append(algorithmic_bytes(nth.cpu(), trainer.texture_dims.cpu(), H, W))
        ab = {k: sum(a[k] for a in abs_) / len(abs_) for k in abs_[0]}

    for w in range(args.warmup):
        if w == 1:
            # twice the first step's transient memory reserved in the caching allocator's pool (allocated and freed at
            # once; the block stays cached): with --warmup < N_POSES a pose with more pairs than any warmup pose is
            # first rendered inside the timed region, where growing the pool (hipMalloc) added 1.2-1.5 ms to that step
            torch.cuda.synchronize()
            transient = torch.cuda.max_memory_allocated(dev) - torch.cuda.memory_allocated(dev)
            torch.empty(2 * transient, dtype=torch.uint8, device=dev)
        step()
    # the last warmup step's deferred texel update stays pending: it is the first kernel of the first timed step (as
    # every step starts with the previous step's texel update), and the last timed step's update runs after the timed
    # region -- K steps, K texel updates, and the first timed step starts with ~90 us of device work queued instead of
    # an idle device waiting for the host's first launches
    carried = trainer._pending_tex is not None  # the first timed step runs the last warmup step's texel update
    # every event recorded into the stream is a marker packet the device waits on (≈ 4 us each, A/B measured), so the
    # timed loop records only what the line needs: one event per step boundary (K + 1, not 2 K) and, at N = 1, the
    # dominant kernel's pair (the raster backward); at N > 1 also the forward's, for the exchange's phase record.
    # The host-side preparation (event creation: ~K hipEventCreate calls) happens here, while the device still runs
    # the warmup's last steps, not after the synchronisation, where the idle device would drop its clock before the
    # timed region
    ops.set_kernel_timing(not args.no_kernel_timing, names=timed)
    if sync is not None and not args.no_kernel_timing:
        sync.phase_events = {}  # when the head / tail collectives land, on rank 0's compute stream
    bound = [_lib.TimingEvent() for _ in range(args.steps + 1)]  # fence-free timing events (`value` is the wall clock)
    host_s = []  # host time to enqueue each step (the device runs behind it when the step is not host-bound)
    base_mb = torch.cuda.memory_allocated(dev) / 2**20  # parameters, Adam state, scene, views, targets
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(dev)
    t0 = time.perf_counter()
    bound[0].record()
    for k in range(args.steps):
        h0 = time.perf_counter()
        step()
        bound[k + 1].record()
        host_s.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    trainer.wait_texture()  # the last timed step's deferred texel update (the first timed step ran the warmup's)
    peak_mb = torch.cuda.max_memory_allocated(dev) / 2**20
    raster_ev = {n: ops._TIMING_EVENTS(n) for n in ("gstex_raster_fwd", "gstex_raster_bwd")}
    kt = ops.kernel_times()
    ops.set_kernel_timing(False)
    step_ms = _events_ms(list(zip(bound[:-1], bound[1:])))
    if world == 1 and not args.no_kernel_timing:
        # the raster forward's launch time from a few untimed steps right after the timed region (same workload)
        ops.set_kernel_timing(True, names={"gstex_raster_fwd"})
        for _ in range(6):
            step()
        trainer.wait_texture()
        kt.update(ops.kernel_times())
        ops.set_kernel_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    mpix = world * H * W / (elapsed / args.steps) / 1e6

    avg = {k: sum(v) / len(v) for k, v in kt.items()}
    med = {k: statistics.median(v) for k, v in kt.items()}
    f_ms = avg.get("gstex_raster_fwd", float("nan"))
    b_ms = avg.get("gstex_raster_bwd", float("nan"))
    dom, dom_ms, dom_bytes = ("raster_bwd", b_ms, ab["bwd"]) if b_ms >= f_ms else ("raster_fwd", f_ms, ab["fwd"])
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    roofline = dict(bound="hbm", kernel=dom, achieved=round(achieved, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(achieved / HBM_PEAK_GBS, 4), traffic=None,
                    traffic_source=f"profiles/{PROFILE_TAG}_traffic.json",
                    bytes_per_launch=int(dom_bytes), launch_ms=round(dom_ms, 4),
                    fwd_bwd_frac=round((ab["fwd"] + ab["bwd"]) / ((f_ms + b_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
    prow = pmc_row(dom)
    if prow is not None:
        # 2 FETCH + WRITE: the gfx950 x2 FETCH_SIZE correction holds for vector loads of every width the kernels use
        # but scalar loads count x1 (profiles/r03_fetch_calibration.json), so with the backward's scalar record reads
        # this is an upper bound; FETCH + WRITE (all loads scalar) is the lower bound
        roofline["traffic"] = int(prow["hbm_bytes_per_launch"])
        if prow.get("fetch_kib") is not None and prow.get("write_kib") is not None:
            roofline["traffic_lower_bound"] = int((prow["fetch_kib"] + prow["write_kib"]) * 1024)
            roofline["traffic_calibration"] = "profiles/r03_fetch_calibration.json"
        if prow.get("valu_insts"):
            # the kernel is VALU-issue/latency bound, not HBM bound: its issue roofline, live time
            roofline["valu_insts_per_launch"] = int(prow["valu_insts"])
            roofline["valu_issue_frac"] = round(prow["valu_insts"] / (dom_ms * 1e-3 * 1024 * 2.4e9 / 2), 4)

    exchange = None
    if sync is not None and sync.phase_events and kt.get("gstex_raster_bwd") and kt.get("gstex_raster_fwd"):
        # per step k: raster bwd end -> head landed -> tail landed (in step k+1's render) -> next raster fwd start
        pe = dict(sync.phase_events)
        if carried and pe.get("tail"):
            # the first timed step's deferred update (and its tail landing) belongs to the last warmup step
            pe["tail"] = pe["tail"][1:]
        bwd, fwd = raster_ev["gstex_raster_bwd"], raster_ev["gstex_raster_fwd"]
        rows = []
        for k in range(min(len(bwd), len(pe.get("head", [])), len(pe.get("tail", [])))):
            if k + 1 >= len(fwd):
                break
            b_end = bwd[k][1]
            rows.append((b_end.elapsed_time(pe["head"][k]), b_end.elapsed_time(pe["tail"][k]),
                         b_end.elapsed_time(fwd[k + 1][0])))
        if rows:
            ph = [round(statistics.median(r[i] for r in rows), 4) for i in range(3)]
            exchange = dict(bytes=int(sync.nbytes), steps=len(rows), bwd_end_to_head_landed_ms=ph[0],
                            bwd_end_to_tail_landed_ms=ph[1], bwd_end_to_next_fwd_ms=ph[2],
                            note="rank 0 HIP events, medians over the timed steps; the exchange's exposed time is "
                                 "bwd_end_to_next_fwd_ms minus the one-GPU gap (DESIGN.md §6)")
        sync.phase_events = None
    sub = None
    if rank == 0 and world == 1 and not args.no_sub:
        sub = {}
        # HBM footprint of the timed steps (torch allocator): resident state, and the peak including the step's
        # transient buffers (pair lists, records, per-pixel state, forward aux / checkpoints, gradients)
        sub["hbm_mb"] = dict(resident=round(base_mb, 1), step_peak=round(peak_mb, 1),
                             step_transient=round(peak_mb - base_mb, 1))
        try:
            # the full-output forward (depth / distortion / normal produced: the reference kernel's contract)
            trainer.geometry_outputs = True
            ops.set_kernel_timing(True)
            with torch.no_grad():
                for _ in range(10):
                    trainer.render(views[0], sh_degree_now=3, composite=False)
            kf = ops.kernel_times()
            ops.set_kernel_timing(False)
            trainer.geometry_outputs = False
            sub["raster_fwd_full_outputs_ms"] = round(statistics.median(kf["gstex_raster_fwd"]), 4)
            sub["eval_render"] = dict(ms_per_image=round(eval_render_ms(trainer, views[0], 10), 4),
                                      reference_raster_calls=3, raster_passes=2, channels=6,
                                      note="gstex.py:1165-1203, no grad; one binning for the three calls, channels "
                                           "3..5 (zero texels) not rasterised, the settings | 1 << 15 call (zero edit "
                                           "texture, unit normals) derived from the first one's outputs "
                                           "(GStexTrainer.eval_render)")
            sub["eval_render"]["fps"] = round(1e3 / sub["eval_render"]["ms_per_image"], 1)
            rc = []
            for _ in range(3):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                trainer.recharge()
                torch.cuda.synchronize()
                rc.append((time.perf_counter() - t1) * 1e3)
            sub["rechart_ms"] = round(statistics.median(rc), 3)
            sub["cfg2_fwd_bwd"] = raster_only(50_000, 1e6, 800, 800, 20, dev)
            sub["cfg1_fwd"] = raster_only(1_000, 0, 256, 256, 50, dev, backward=False)
            # cfg5's per-GPU raster: one 1600x1200 view with depth + normal outputs and gradients (the DTU scan24
            # COLMAP init is absent: a synthetic scene of the bench's size stands in)
            sub["cfg5_fwd_bwd_geo"] = raster_only(200_000, 1e7, 1200, 1600, 10, dev, geo=True)
        except Exception as ex:  # sub-records must never kill the headline line
            sub["error"] = repr(ex)

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        th = cpu_threads()
        try:
            cpu = cpu_baseline(make_scene(args.n_splats, args.n_texels, seed=args.seed), sphere_view(0, H, W),
                               args.cpu_crop, th)
            if sub is not None:
                torch.set_num_threads(th)
                sc1 = make_scene(1_000, 0, seed=42)
                t1 = [oracle_crop(sc1, sphere_view(0, 256, 256), 256, bwd=False) for _ in range(3)]
                sub["cfg1_fwd"]["cpu_oracle_ms_median"] = round(1e3 * statistics.median(t1), 1)
                sc2 = make_scene(50_000, 1e6, seed=42)
                t2 = oracle_crop(sc2, sphere_view(0, 800, 800), 128)
                sub["cfg2_fwd_bwd"]["cpu_oracle_128x128_crop_s"] = round(t2, 2)
        except Exception as ex:  # baseline must never kill the GPU result line
            cpu = dict(value=None, unit="Mpix/s", cores=th, kind="port", sample=f"failed: {ex!r}")
    line = {
        "metric": "train-step ms + rendered Mpix/s, 200k splats/1e7 texels @800x800",
        "value": round(mpix, 4),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "ms_per_step_median": round(statistics.median(step_ms), 4),
        "step_ms_events": [round(x, 3) for x in step_ms],  # rank 0's per-step HIP-event times
        "host_enqueue_ms_median": round(1e3 * statistics.median(host_s), 4),  # Python + launch time per step
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seed 42 random-init splats, charted random texels, random target images)",
        "config": {
            "workload": "cfg3 full GStex train step (fwd+loss+bwd+Adam), one 800x800 view per GPU per step",
            "n_splats": args.n_splats, "n_texels": int(trainer.n_texels), "H": H, "W": W,
            "views_per_step": world, "parallelism": f"dp{world}",
            "cameras": f"rank r, step s: pose (r + s*N) mod {N_POSES} of {N_POSES} fixed sphere poses",
            "stationary": "means/scales/quats/opacity logits restored before every step (timed); colours, texels "
                          "and Adam moments train",
            "sh_degree": trainer.sh_degree_now(), "settings": trainer.settings,
            "geometry_outputs": trainer.geometry_outputs,
            "fold_aabb": True, "texture_transform": "SH2RGB on read (0.28209479, 0.5)",
            "pair_buffers": ("capacity-sized, pair total kept on the device: no host read-back or synchronisation in "
                             "the step (ops.PairCapacity, capacity %d)" % trainer.pairs.capacity
                             if trainer.pairs is not None else "sized by a host read-back of the pair total"),
            "step_launch": ("eager: every launch enqueued by the host each step" +
                            ("; the render's launches before the raster forward as one C call and the render as one "
                             "autograd node (gstex_amd.fused)" if trainer.fused_step else "")),
            "texture_update": ("deferred: step k's texel Adam update is the first kernel of step k+1 (same stream, "
                                    "before the raster forward); the timed region holds exactly K texel updates "
                                    "(the last warmup step's and those of timed steps 1..K-1)"
                               if trainer.defer_texture
                               else "compute stream"),
        },
        "roofline": roofline,
        "cpu_baseline": cpu,
        "kernel_ms": {k.replace("gstex_", ""): round(v, 4) for k, v in avg.items()},
        "kernel_ms_median": {k.replace("gstex_", ""): round(v, 4) for k, v in med.items()},
        "counts": {k: int(ab[k]) for k in ("N_v", "I", "T_v", "P")},
        "sub": sub,
        "exchange": exchange,
        "setup_s": round(setup_s, 1),
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
