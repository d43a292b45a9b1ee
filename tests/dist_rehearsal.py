#!/usr/bin/env python3
"""Multi-rank rehearsal of the REAL data-parallel training path on one GPU (test infrastructure).

    GSTEX_DIST_BACKEND=gloo torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \\
        tests/dist_rehearsal.py [--steps 3] [--n-splats 200000 --n-texels 1e7 --size 800] [--defer-texture] [--geo]

Launched by tests/test_gpu_dist.py as a fresh child process (torch.distributed.run), and by hand for other sizes.
Every rank runs GStexTrainer + GradSync + the HIP kernels on cuda:0 (the pool's boxes have one GPU; gloo carries the
collectives through host memory, RCCL needs one GPU per rank).  Per step, rank r renders its own camera pose
(r + step * world) mod 8 -- the cfg4 sharding of camera views (reference: one camera per rank and step,
scripts/train.py:97,138-144; DDP averaging, pipelines/base_pipeline.py:281-283).  Exercised:
  * the raster backward accumulating the texel gradient into the flat buffer's slice (the sink) and the exchange:
    the plain all_reduce() in step 0, the overlapped one inside GStexTrainer.optimizer_step(sync=...) after it --
    tail started from the raster backward, or with --defer-texture head first, the tail in GradSync.tail_bounds
    pieces, each stepped by FusedAdam.step_range as it lands, inside the next step's render;
  * step 1: trainer.zero_grad() (set_to_none) AFTER sync.zero() -- autograd writes detached .grad tensors, which the
    exchange must fold back into the buffer;
  * after step 1: a rechart that GROWS the texel store (new Parameter, new flat buffer and sink at the next zero()).

The check is on the GRADIENT each Adam launch consumes: every FusedAdam.step /
step_range call of the data-parallel trainer is intercepted and the gradient it reads (times its grad_scale, i.e. the
all-reduced mean gradient) is recorded per parameter group and step; rank 0 runs a single-rank reference trainer on
the same `world` views per step (autograd sums them, the sum is scaled by 1/world) with its parameters set to the
data-parallel trainer's before every step ("mirrored": each step compares gradients taken at identical parameters), and
a second mirrored reference gives the run-to-run floor of the float-atomic sums.  Pass:
  * every group, every step: ||g_dist - g_ref|| / ||g_ref|| <= 1e-5 (and printed next to the floor
    ||g_ref2 - g_ref|| / ||g_ref||); a wrong 1/world factor, a dropped or doubled piece, or a stale sink shows up
    as an error of order 1;
  * with --deterministic (torch.use_deterministic_algorithms: splat-gradient rows summed in a fixed order)
    at world 2, the splat groups bit-exact at every step (a + b == b + a);
  * every rank's parameters equal rank 0's bit for bit after the run.
Parameters of rank 0 vs a FREE-running single-rank reference (its own mean-gradient Adam steps) are reported, not
asserted: Adam (eps 1e-15) moves an element by ~lr whatever its gradient's size, so a texel whose gradient is
float-atomic noise around zero differs by up to 2 lr per step between ANY two runs (shown for the worst texel: its
per-step gradients in both runs next to the median |gradient|) -- the mechanism behind round 3's geo4 "failure".
Prints one line per check and `REHEARSAL OK world=N` at the end (exit status 0), else `REHEARSAL FAILED`.
"""
import argparse
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_POSES = 8


class AdamTap:
    """Records the gradient every FusedAdam launch of `trainer` consumes: {group name: [per-step fp32 tensors]}."""

    def __init__(self, trainer):
        self.tr = trainer
        self.grads = {}
        self._piece = {}
        opt = trainer.optimizer
        step, step_range = opt.step, opt.step_range

        def names():
            return {id(p): n for n, p in zip(trainer.param_groups(), trainer.parameters())}

        def tap_step(closure=None, only=None, skip=None, grad_scale=1.0, **kw):
            nm = names()
            for p in trainer.parameters():
                if p.grad is None or (only is not None and id(p) not in only) or (skip is not None and id(p) in skip):
                    continue
                self.grads.setdefault(nm[id(p)], []).append((p.grad * grad_scale).detach().clone())
            return step(closure=closure, only=only, skip=skip, grad_scale=grad_scale, **kw)

        def tap_range(p, lo, hi, first, grad_scale=1.0, **kw):
            name = names()[id(p)]
            if first:
                self._piece[name] = torch.full_like(p.grad, float("nan"))
                self.grads.setdefault(name, []).append(self._piece[name])
            self._piece[name].view(-1)[lo:hi] = p.grad.view(-1)[lo:hi] * grad_scale
            return step_range(p, lo, hi, first, grad_scale=grad_scale, **kw)

        opt.step = tap_step
        opt.step_range = tap_range


def mirror(ref, tr):
    """Set reference trainer `ref` to `tr`'s parameters and charts (its own Adam state is never used)."""
    with torch.no_grad():
        if ref.texture_dc.shape != tr.texture_dc.shape:  # tr's texel store grew at a rechart
            old = ref.texture_dc
            ref.texture_dc = torch.nn.Parameter(tr.texture_dc.detach().clone())
            for g in ref.optimizer.param_groups:
                if g["name"] == "texture_dc":
                    g["params"] = [ref.texture_dc]
            ref.optimizer.state.pop(old, None)
        ref.texture_dims = tr.texture_dims.clone()
        ref.mappings.copy_(tr.mappings)
        ref.n_texels = tr.n_texels
        for p, q in zip(ref.parameters(), tr.parameters()):
            p.copy_(q.detach())


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm()) / max(float(b.norm()), 1e-300)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--n-splats", type=int, default=20_000)
    ap.add_argument("--n-texels", type=float, default=4e5)
    ap.add_argument("--size", type=int, default=160, help="square image side (ignored with --height/--width)")
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--geo", action="store_true",
                    help="cfg5's training mode: depth / distortion / normal rendered and regularised (lambda_normal 0.05, "
                         "lambda_reg 0.01, use_normal_loss: the geometry backward under the exchange)")
    ap.add_argument("--defer-texture", action="store_true",
                    help="GStexTrainer(defer_texture=True): the texel update of step k runs in step k+1's render")
    ap.add_argument("--deterministic", action="store_true",
                    help="torch.use_deterministic_algorithms(True): splat-gradient rows summed in a fixed order")
    args = ap.parse_args()
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    dist.init_process_group(os.environ.get("GSTEX_DIST_BACKEND", "gloo"), init_method="env://")
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    if args.deterministic:
        torch.use_deterministic_algorithms(True, warn_only=True)

    from gstex_amd.dist import GradSync
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    H = args.height or args.size
    W = args.width or args.size
    sc = make_scene(args.n_splats, args.n_texels, seed=11)
    views = [sphere_view(i, H, W, n_views=N_POSES).to(dev) for i in range(N_POSES)]
    g = torch.Generator().manual_seed(2024)
    gts = [torch.rand((H, W, 3), generator=g).to(dev) for _ in range(N_POSES)]
    geo = dict(lambda_normal=0.05, lambda_reg=0.01, use_normal_loss=True) if args.geo else {}
    tr = GStexTrainer(sc, dev, start_step=3000, defer_texture=args.defer_texture, **geo)
    sync = GradSync(tr, world)
    tap = AdamTap(tr)
    # rank 0: two MIRRORED references (their parameters set to the data-parallel trainer's before each step's
    # gradients, so every step compares gradients at identical inputs; the second one gives the float-atomic floor)
    # and one FREE-running reference that steps its own Adam (the parameter-level report)
    refs = [GStexTrainer(sc, dev, start_step=3000, **geo) for _ in range(2)] if rank == 0 else []
    free = GStexTrainer(sc, dev, start_step=3000, **geo) if rank == 0 else None
    ref_grads = [{} for _ in refs]
    free_tap = AdamTap(free) if free is not None else None

    def say(msg):
        if rank == 0:
            print(msg, flush=True)

    def agree(flag: bool) -> bool:
        t = torch.tensor([1.0 if flag else 0.0], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item() == 1.0)

    say(f"world {world}, {args.n_splats} splats, {args.n_texels:.3g} texels, {W}x{H}, steps {args.steps}, "
        f"defer_texture {tr.defer_texture}, geo {args.geo}, deterministic {args.deterministic}, "
        f"backend {dist.get_backend()}")
    ok = True
    for step in range(args.steps):
        pose = (rank + step * world) % N_POSES
        sync.zero()
        if step == 1:
            tr.zero_grad()  # set_to_none after zero(): detached autograd .grad tensors, folded back by the exchange
        tr.forward_backward(views[pose], gts[pose])
        # the parameters this step's gradients were taken at: the head groups as the last step left them, the texels
        # after the deferred update the render above ran
        for ref in refs:
            mirror(ref, tr)
        # the tail's collective starts from the raster backward -- unless the exchange is head first (a deferring
        # trainer), where the step queues it behind the head's
        started = (sync._work is not None) != sync.head_first
        if step == 0:  # the plain exchange: averaged gradient buffer, then the step
            sync.all_reduce()
            tr.optimizer_step()
        else:  # the overlapped exchange inside the step (1/world in the fused update)
            tr.optimizer_step(sync=sync)
        flag = agree(started)
        say(f"step {step}: poses {[(r + step * world) % N_POSES for r in range(world)]}, tail collective "
            + ("queued behind the head's (head first)" if sync.head_first else "started from the raster backward")
            + f" on every rank: {flag}")
        ok &= flag
        for ref, rg in zip(refs + ([free] if free is not None else []), ref_grads + [None]):
            ref.zero_grad()
            for r in range(world):
                p = (r + step * world) % N_POSES
                ref.forward_backward(views[p], gts[p])  # autograd accumulates the world gradients (sum)
            for name, prm in zip(ref.param_groups(), ref.parameters()):
                if prm.grad is not None:
                    prm.grad.mul_(1.0 / world)  # the mean gradient
                    if rg is not None:
                        rg.setdefault(name, []).append(prm.grad.detach().clone())
            if rg is None:
                ref.optimizer_step()
        if step == 1:
            old = tr.texture_dc
            cap = old.shape[0]
            for t in [tr] + ([free] if free is not None else []):
                t.pixel_num = 1.3 * cap  # the new charts need more texels than the store holds: it grows
                t.recharge()
            grew = tr.texture_dc is not old and tr.texture_dc.shape[0] > cap
            say(f"rechart after step 1: texel store {cap} -> {tr.texture_dc.shape[0]} rows "
                f"(new Parameter: {tr.texture_dc is not old}), n_texels {tr.n_texels}")
            ok &= agree(grew)
    tr.wait_texture()  # a deferred texel update still pending after the last step
    torch.cuda.synchronize()

    # 1. the gradient every Adam launch consumed, vs the single-rank mean gradient
    names = list(tr.param_groups())
    good = True
    worst_tex = None
    if rank == 0:
        say("gradient consumed by Adam, ||g_dist - g_ref|| / ||g_ref|| per step (floor: a second reference run):")
        for name in names:
            gd, gr, g2 = tap.grads.get(name, []), ref_grads[0].get(name, []), ref_grads[1].get(name, [])
            if not gr and not g2 and len(gd) == args.steps and all(float(t.abs().max()) == 0.0 for t in gd):
                # a parameter no rank takes a gradient for (features_dc under SH colour, gstex.py:1100): its slice of the
                # flat buffer is reduced as zeros (DDP's find_unused_parameters) and Adam's update of it is exactly 0
                say(f"  {name:14s} unused: all-zero reduced gradient (no-op update), reference: no gradient")
                continue
            if not (len(gd) == len(gr) == len(g2) == args.steps):
                say(f"  {name:14s} launches: dist {len(gd)}, ref {len(gr)}, ref2 {len(g2)} (expected {args.steps})"
                    "   <-- FAIL")
                good = False
                continue
            errs, floors = [], []
            for a, b, c in zip(gd, gr, g2):
                if a.shape != b.shape or bool(torch.isnan(a).any()):
                    errs.append(float("inf"))
                    continue
                errs.append(rel(a, b))
                floors.append(rel(c, b))
            line = (f"  {name:14s} " + " ".join(f"{e:.2e}" for e in errs) + "   floor "
                    + " ".join(f"{f:.2e}" for f in floors))
            g_ok = max(errs) <= 1e-5
            if args.deterministic and world == 2 and name != "texture_dc":
                exact = all(bool(torch.equal(a, b)) for a, b in zip(gd, gr))
                line += f"   bit-exact {exact}"
                g_ok &= exact
            good &= g_ok
            say(line + ("" if g_ok else "   <-- FAIL"))
        worst_tex = (tap.grads.get("texture_dc"), free_tap.grads.get("texture_dc"))
    ok &= agree(good)

    # 2. every rank equals rank 0 bit for bit; rank 0 vs the reference (reported; see the module docstring)
    for name, prm in zip(names, tr.parameters()):
        mine = prm.detach().clone()
        r0 = mine.clone()
        dist.broadcast(r0, 0)
        same = agree(bool(torch.equal(mine, r0)))
        ok &= same
        line = f"{name:14s} every rank == rank 0: {same}"
        if rank == 0:
            rp = dict(zip(free.param_groups(), free.parameters()))[name].detach()
            if rp.shape != r0.shape:
                # the free-running reference recharted from its own parameters, which differ from rank 0's by float
                # rounding (order of the float atomics): a splat whose chart size is an integer step function of its
                # scale can land on the other side of a step, so the texel stores differ in length -- reported only
                say(line + f";  free-running reference recharted to {tuple(rp.shape)} vs {tuple(r0.shape)} (not compared)")
                continue
            scale = max(float(rp.abs().max()), 1e-30)
            d = (r0 - rp).abs()
            lr = free.optimizer.param_groups[names.index(name)]["lr"]
            line += f";  |rank0 - free-running reference| max {float(d.max()) / scale:.2e}, mean {float(d.mean()) / scale:.2e} of max|p|"
            line += f" (worst element {float(d.max()) / lr:.2f} lr)"
            if name == "texture_dc" and worst_tex is not None and worst_tex[0] is not None:
                i = int(torch.argmax(d.reshape(-1)))
                gd = [float(t.reshape(-1)[i]) if t.numel() > i else float("nan") for t in worst_tex[0]]
                gr = [float(t.reshape(-1)[i]) if t.numel() > i else float("nan") for t in worst_tex[1]]
                med = float(worst_tex[1][-1].abs().reshape(-1)[worst_tex[1][-1].reshape(-1) != 0].median())
                line += (f"\n    worst texel element {i}: gradient per step dist {['%.2e' % v for v in gd]}, "
                         f"ref {['%.2e' % v for v in gr]}; median |gradient| {med:.2e}")
        say(line)
    say(f"flat buffer {sync.nbytes / 1e6:.1f} MB")
    say(("REHEARSAL OK" if ok else "REHEARSAL FAILED") + f" world={world}")
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
