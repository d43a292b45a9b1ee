"""Shared case builders: one seeded synthetic case evaluated by the CPU oracle and by the HIP path."""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from gstex_amd.scene import make_scene, sphere_view
from oracle import raster as O

TOL_ABS = 1e-5  # forward parity tolerance (fp32), north_star: "within 1e-5 fp32"
TOL_REL = 1e-5
GRAD_RTOL = 1e-5  # gradient tolerance (norm-wise and max-element relative, vs the oracle's fp64 autograd), test_gpu_parity.py


@dataclass
class Case:
    inp: O.RasterInputs
    view: object
    C: int
    nth: torch.Tensor
    flip_mask: torch.Tensor = None  # set by oracle_run: pixels excluded from gradient comparisons


def make_case(n=300, n_texels=20000, H=64, W=80, seed=0, view=0, opacity=None, C=3,
              settings=(1 << 9) | (1 << 10), bg=None, cube=2.0, glob_scale=1.0):
    sc = make_scene(n, n_texels, channels=C, seed=seed, opacity=opacity, cube=cube)
    v = sphere_view(view, H, W)
    means, scales, quats, opac = sc.activated()
    cam = O.Camera(v.viewmat, v.fx, v.fy, v.cx, v.cy, H, W, 16, v.c2w[:3, 3])
    centers, extents = O.aabb_2d(means, scales, glob_scale, quats, cam)
    _, depths = O.project_points(means, cam)
    nth = O.num_tiles_hit(centers, extents, H, W)
    uv0, umap, vmap = sc.uv_mapping()
    g = torch.Generator().manual_seed(seed + 1000)
    rgbs = torch.rand((n, 3), generator=g)
    inp = O.RasterInputs(sc.texture_dims, centers.detach().clone(), extents, depths, rgbs, opac.detach().clone(),
                         means.detach().clone(), scales.detach().clone(), glob_scale, quats.detach().clone(),
                         uv0.detach().clone(), umap, vmap, sc.texture.clone(), cam, settings,
                         None if bg is None else torch.tensor(bg, dtype=torch.float32))
    return Case(inp, v, C, nth)


DIFF = ["rgbs", "opacities", "means", "scales", "quats", "texture", "centers", "uv0"]


def upstream(H, W, C, seed=5, mask=None):
    """Seeded upstream gradients of the six outputs; zero at the pixels of `mask` (H, W bool) if given."""
    g = torch.Generator().manual_seed(seed)
    up = dict(img=torch.randn(H, W, 3, generator=g), depth=torch.randn(H, W, generator=g),
              reg=torch.randn(H, W, generator=g), alpha=torch.randn(H, W, generator=g),
              tex=torch.randn(H, W, C, generator=g), normal=torch.randn(H, W, 3, generator=g))
    if mask is not None and bool(mask.any()):
        for k, v in up.items():
            v[mask] = 0.0
    return up


def _differentiable(settings, outputs):
    """Outputs that take an upstream gradient: with settings bit 15 the unit normal is a forward-only output."""
    if settings & O.SETTING_EVAL_NORMAL:
        names = outputs if outputs is not None else ("img", "depth", "reg", "alpha", "tex", "normal")
        return tuple(k for k in names if k != "normal")
    return outputs


def oracle_run(case: Case, grads=True, seed=5, grad_dtype=torch.float64, outputs=None, flip_mask=None):
    """flip_mask: use this mask (e.g. one computed on another machine, whose CPU exp may round differently) instead of
    the one this run's margins give."""
    inp = case.inp
    leaves = {}
    if grads:
        for k in DIFF:
            t = getattr(inp, k).detach().clone().requires_grad_(True)
            setattr(inp, k, t)
            leaves[k] = t
    o32, o64, aux = O.rasterize(inp, grad_dtype=grad_dtype)
    # pixels with a threshold decision within FLIP_MARGIN (an exp ulp may flip it on the GPU; the forward check
    # accounts for them) take no upstream gradient in either run, so a flipped pair cannot enter the comparison
    case.flip_mask = aux["margin"] < FLIP_MARGIN if flip_mask is None else flip_mask
    out = {}
    outputs = _differentiable(inp.settings, outputs)
    if grads:
        up = upstream(inp.cam.H, inp.cam.W, case.C, seed, case.flip_mask)
        loss = sum((o64[k] * up[k].to(grad_dtype)).sum() for k in up if outputs is None or k in outputs)
        loss.backward()
        out = {k: (v.grad.detach().clone() if v.grad is not None else torch.zeros_like(v).detach()).float()
               if v.grad is None else v.grad.detach().clone() for k, v in leaves.items()}
        for k in DIFF:
            setattr(inp, k, getattr(inp, k).detach())
    return o32, o64, aux, out


def gpu_run(case: Case, grads=True, seed=5, device="cuda", outputs=None):
    """outputs: names of the outputs that receive an upstream gradient (default all six; the others
    reach the kernel as NULL, as for outputs the loss does not use)."""
    import gstex_cuda

    inp = case.inp
    v = case.view
    dv = lambda t: t.detach().to(device).contiguous()  # noqa: E731
    t = {k: dv(getattr(inp, k)) for k in DIFF}
    if grads:
        for k in t:
            t[k].requires_grad_(True)
    n = inp.means.shape[0]
    outs = gstex_cuda.texture_gaussians(
        (n, 1, case.C), dv(inp.texture_dims), t["centers"], dv(inp.extents), dv(inp.depths), dv(case.nth),
        t["rgbs"], t["opacities"], t["means"], t["scales"], inp.glob_scale, t["quats"], t["uv0"], dv(inp.umap),
        dv(inp.vmap), t["texture"], dv(v.viewmat), dv(v.c2w), v.fx, v.fy, v.cx, v.cy, inp.cam.H, inp.cam.W, 16,
        inp.settings, background=None if inp.background is None else dv(inp.background))
    names = ["img", "depth", "reg", "alpha", "tex", "normal"]
    res = {k: o.detach().cpu() for k, o in zip(names, outs)}
    gr = {}
    outputs = _differentiable(inp.settings, outputs)
    if grads:
        up = upstream(inp.cam.H, inp.cam.W, case.C, seed, case.flip_mask)
        sel = [i for i, k in enumerate(names) if outputs is None or k in outputs]
        torch.autograd.backward([outs[i] for i in sel], [up[names[i]].to(device) for i in sel])
        gr = {k: (t[k].grad.detach().cpu() if t[k].grad is not None else torch.zeros_like(t[k]).cpu()) for k in t}
    return res, gr


FLIP_MARGIN = 1e-5  # relative distance from a threshold within which an fp32 decision may flip (exp/rcp ulps)
FLIP_FRACTION = 1e-3  # at most this fraction of the pixels (and at least 4) may carry a flipped decision


def assert_close_fwd(gpu, ref64, names=("img", "depth", "reg", "alpha", "tex", "normal"), margin=None):
    """Every output element within 1e-5 (+1e-5 relative) of the oracle.  With `margin` (the oracle's per-pixel
    decision margins, aux["margin"]): a pixel outside the tolerance passes only if one of its threshold decisions
    lies within FLIP_MARGIN of the threshold (an ulp of exp can flip it on either side), and such pixels are
    rare (FLIP_FRACTION)."""
    flipped = None
    for k in names:
        a = gpu[k].double()
        b = ref64[k].double()
        err = (a - b).abs()
        bound = TOL_ABS + TOL_REL * b.abs()
        bad = err > bound
        if margin is not None and bool(bad.any()):
            pix = bad if bad.dim() == 2 else bad.any(-1)
            unexplained = pix & ~(margin < FLIP_MARGIN)
            assert not bool(unexplained.any()), (
                f"{k}: {int(unexplained.sum())} pixels outside 1e-5 (+1e-5 rel) with no decision near a threshold; "
                f"max err {err.max().item():.3e}")
            flipped = pix if flipped is None else flipped | pix
            continue
        assert not bool(bad.any()), (
            f"{k}: {int(bad.sum())} / {bad.numel()} elements outside 1e-5 (+1e-5 rel); max err {err.max().item():.3e}")
    if flipped is not None:
        n = int(flipped.sum())
        assert n <= max(4, FLIP_FRACTION * flipped.numel()), f"{n} pixels with flipped decisions"
        print(f"[parity] {n} / {flipped.numel()} pixels differ by a decision flipped within {FLIP_MARGIN:g} of its threshold")


def grad_rel_err(g, ref):
    if ref.numel() == 0:
        return 0.0, 0.0
    scale = ref.abs().max().item()
    return (g.double() - ref.double()).abs().max().item() / max(scale, 1e-12), scale


def grad_norm_err(g, ref):
    if ref.numel() == 0:
        return 0.0
    n = ref.double().norm().item()
    return (g.double() - ref.double()).norm().item() / max(n, 1e-30)


_SCENES: dict = {}


def make_window_case(n, n_texels, H, W, win, seed=42, view=0, C=3, settings=(1 << 9) | (1 << 10), opacity=0.1):
    """A win x win window at the centre of the H x W sphere view `view` of the seeded make_scene(n, n_texels)
    (the bench scenes: cfg3 = 200k / 1e7 / 800x800, cfg2 = 50k / 1e6 / 800x800): the camera's principal point
    is shifted by the window origin (the bench's cpu_baseline crop), and only the splats that reach the window
    are kept, their texel blocks repacked contiguously (same texels, offsets re-based) -- the other splats
    contribute nothing to these pixels.  Returns a Case usable by oracle_run / gpu_run."""
    from gstex_amd.scene import View

    key = (n, n_texels, seed, opacity)
    if key not in _SCENES:
        _SCENES.clear()
        _SCENES[key] = make_scene(n, n_texels, channels=C, seed=seed, opacity=opacity)
    sc = _SCENES[key]
    full = sphere_view(view, H, W)
    x0, y0 = W // 2 - win // 2, H // 2 - win // 2
    v = View(full.viewmat, full.c2w, full.fx, full.fy, full.cx - x0, full.cy - y0, win, win)
    means, scales, quats, opac = sc.activated()
    cam = O.Camera(v.viewmat, v.fx, v.fy, v.cx, v.cy, win, win, 16, v.c2w[:3, 3])
    centers, extents = O.aabb_2d(means, scales, 1.0, quats, cam)
    nth = O.num_tiles_hit(centers, extents, win, win)
    keep = torch.nonzero(nth > 0).squeeze(1)
    dims = sc.texture_dims[keep].clone()
    hw = (dims[:, 0].long() * dims[:, 1].long())
    rows = torch.cat([torch.arange(int(o), int(o) + int(s)) for o, s in zip(sc.texture_dims[keep, 2].tolist(),
                                                                            hw.tolist())]) if keep.numel() else \
        torch.zeros(0, dtype=torch.long)
    dims[:, 2] = (torch.cumsum(hw, 0) - hw).to(torch.int32)
    texture = sc.texture[rows].clone() if rows.numel() else torch.zeros((0, C))
    uv0, umap, vmap = sc.uv_mapping()
    means, scales, quats, opac = means[keep], scales[keep], quats[keep], opac[keep]
    _, depths = O.project_points(means, cam)
    g = torch.Generator().manual_seed(seed + 1000)
    rgbs = torch.rand((sc.n, 3), generator=g)[keep]
    inp = O.RasterInputs(dims, centers[keep].detach().clone(), extents[keep], depths, rgbs,
                         opac.detach().clone(), means.detach().clone(), scales.detach().clone(), 1.0,
                         quats.detach().clone(), uv0[keep].detach().clone(), umap[keep], vmap[keep], texture, cam,
                         settings, None)
    return Case(inp, v, C, nth[keep])
