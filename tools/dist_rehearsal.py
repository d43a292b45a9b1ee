#!/usr/bin/env python3
"""Multi-rank rehearsal of the REAL data-parallel training path on one GPU.

    GSTEX_DIST_BACKEND=gloo torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \\
        tools/dist_rehearsal.py [--steps 3]

Every rank runs GStexTrainer + GradSync + the HIP kernels on cuda:0 (the pool's boxes have one GPU; gloo carries
the collective through host memory, RCCL needs one GPU per rank).  Per step, rank r renders its own camera pose
(r + step * world) mod 8 -- the cfg4 sharding of camera views (reference: one random camera per rank
and step, scripts/train.py:97, full_images_datamanager.py:320, DDP averaging pipelines/base_pipeline.py:281-283).
Exercised, per step:
  * the raster backward accumulating the texel gradient into the flat buffer's slice (the sink) and the tail
    collective started from on_texture_grad (asserted: GradSync._work is set before all_reduce());
  * the head all-reduce, 1/world averaging, the 7-group FusedAdam; from step 1 on the overlapped exchange inside
    GStexTrainer.optimizer_step(sync=...) (texel group updated while the head collective runs, 1/world in the update);
  * step 1: trainer.zero_grad() (set_to_none) AFTER sync.zero() -- autograd then writes detached .grad tensors,
    which all_reduce() must fold back into the buffer;
  * after step 1: a rechart that GROWS the texel store (new Parameter, new flat buffer and sink at the next zero()).
Checked on rank 0 against a single-rank reference trainer that runs the same `world` views per step, sums their
gradients by autograd accumulation, scales by 1/world and takes the same Adam step (the mean-gradient step); every
rank's parameters must equal rank 0's.  Tolerance: 1e-5 of each parameter's max magnitude; for the texels (float-
atomic gradient sums whose order varies run to run, through Adam's m / sqrt(v)) the worst texel within two learning
rates per step (a near-zero gradient's noise of either sign moves it by up to lr) and the mean difference within 1e-6
of the max magnitude.
Test infrastructure; prints one line per check and `REHEARSAL OK world=N` at the end.
"""
import argparse
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_POSES = 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--n-splats", type=int, default=20_000)
    ap.add_argument("--n-texels", type=float, default=4e5)
    ap.add_argument("--size", type=int, default=160)
    ap.add_argument("--geo", action="store_true",
                    help="cfg5's training mode: depth / distortion / normal rendered and regularised (lambda_normal 0.05, "
                         "lambda_reg 0.01, use_normal_loss: the geometry backward under the exchange)")
    ap.add_argument("--defer-texture", action="store_true",
                    help="GStexTrainer(defer_texture=True): the texel update of step k runs in step k+1's render")
    args = ap.parse_args()
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    dist.init_process_group(os.environ.get("GSTEX_DIST_BACKEND", "gloo"), init_method="env://")
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)

    from gstex_amd.dist import GradSync
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    S = args.size
    sc = make_scene(args.n_splats, args.n_texels, seed=11)
    views = [sphere_view(i, S, S, n_views=N_POSES).to(dev) for i in range(N_POSES)]
    g = torch.Generator().manual_seed(2024)
    gts = [torch.rand((S, S, 3), generator=g).to(dev) for _ in range(N_POSES)]
    geo = dict(lambda_normal=0.05, lambda_reg=0.01, use_normal_loss=True) if args.geo else {}
    tr = GStexTrainer(sc, dev, start_step=3000, defer_texture=args.defer_texture, **geo)
    sync = GradSync(tr, world)
    ref = GStexTrainer(sc, dev, start_step=3000, **geo) if rank == 0 else None
    log = []

    def say(msg):
        if rank == 0:
            print(msg, flush=True)
            log.append(msg)

    ok = True
    for step in range(args.steps):
        pose = (rank + step * world) % N_POSES
        sync.zero()
        if step == 1:
            tr.zero_grad()  # set_to_none after zero(): detached autograd .grad tensors, folded back by all_reduce()
        tr.forward_backward(views[pose], gts[pose])
        # the tail's collective starts from the raster backward -- unless the exchange is head first (a deferring
        # trainer), where the step queues it behind the head's
        started = (sync._work is not None) != sync.head_first
        if step == 0:  # the plain exchange: averaged gradient buffer, then the step
            sync.all_reduce()
            tr.optimizer_step()
        else:  # the overlapped exchange inside the step (texel update during the head collective, 1/world in Adam)
            tr.optimizer_step(sync=sync)
        flags = torch.tensor([1.0 if started else 0.0], device=dev)
        dist.all_reduce(flags, op=dist.ReduceOp.MIN)
        say(f"step {step}: poses {[(r + step * world) % N_POSES for r in range(world)]}, tail collective "
            + ("queued behind the head's (head first)" if sync.head_first else "started from the raster backward")
            + f" on every rank: {bool(flags.item() == 1.0)}")
        ok &= bool(flags.item() == 1.0)
        if ref is not None:
            ref.zero_grad()
            for r in range(world):
                p = (r + step * world) % N_POSES
                ref.forward_backward(views[p], gts[p])  # autograd accumulates the world gradients (sum)
            for prm in ref.parameters():
                if prm.grad is not None:
                    prm.grad.mul_(1.0 / world)
            ref.optimizer_step()
        if step == 1:
            old = tr.texture_dc
            cap = old.shape[0]
            for t in ([tr] + ([ref] if ref is not None else [])):
                t.pixel_num = 1.3 * cap  # the new charts need more texels than the store holds: it grows
                t.recharge()
            grew = tr.texture_dc is not old and tr.texture_dc.shape[0] > cap
            say(f"rechart after step 1: texel store {cap} -> {tr.texture_dc.shape[0]} rows "
                f"(new Parameter: {tr.texture_dc is not old}), n_texels {tr.n_texels}")
            ok &= grew
    tr.wait_texture()  # a deferred texel update (--defer-texture) still pending after the last step
    torch.cuda.synchronize()
    # every rank equals rank 0; rank 0 equals the single-rank mean-gradient reference
    for name, prm in zip([n for n in tr.param_groups()], tr.parameters()):
        mine = prm.detach().clone()
        r0 = mine.clone()
        dist.broadcast(r0, 0)
        scale = max(float(r0.abs().max()), 1e-30)
        d_rank = torch.tensor([float((mine - r0).abs().max()) / scale], device=dev)
        dist.all_reduce(d_rank, op=dist.ReduceOp.MAX)
        line = f"{name:14s} max |rank - rank0| / max|p| = {d_rank.item():.2e}"
        good = d_rank.item() < 1e-5
        if ref is not None:
            rp = dict(zip(ref.param_groups(), ref.parameters()))[name].detach()
            d_ref = float((r0 - rp).abs().max()) / scale
            line += f",  |rank0 - mean-gradient reference| / max|p| = {d_ref:.2e}"
            if name == "texture_dc":
                # texel gradients are float-atomic sums (summation order varies run to run) and Adam's m / sqrt(v)
                # (eps 1e-15) turns a near-zero gradient's noise into an update of up to lr either way per step: bound
                # the worst texel by 2 lr per step (the two runs' noise of opposite sign) and the mean by 1e-6 of max|p|
                d_mean = float((r0 - rp).abs().mean()) / scale
                d_abs = float((r0 - rp).abs().max())
                lr = ref.optimizer.param_groups[-1]["lr"]
                line += f" (mean {d_mean:.2e}; worst {d_abs / lr:.2f} lr)"
                good &= d_abs <= 2 * args.steps * lr and d_mean < 1e-6
            else:
                good &= d_ref < 1e-5
        flag = torch.tensor([1.0 if good else 0.0], device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok &= bool(flag.item() == 1.0)
        say(line + ("" if flag.item() == 1.0 else "   <-- FAIL"))
    say(f"flat buffer {sync.nbytes / 1e6:.1f} MB, backend {dist.get_backend()}, world {world}, {args.steps} steps, "
        f"defer_texture {tr.defer_texture}")
    say(("REHEARSAL OK" if ok else "REHEARSAL FAILED") + f" world={world}")
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
