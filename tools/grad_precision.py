#!/usr/bin/env python3
"""Where does the fp32 error of the means / quats gradients arise?  (VERDICT r02 next #4.)

Runs the CPU oracle's autograd on a window of a bench scene in three precision mixes and reports each
gradient's norm-wise and max relative error against the all-fp64 evaluation:
  fp32        per-splat table (the chain raster.hip's setup / setup_bwd implement) and per-pair part in fp32
              (--fp32-record: the round-2 formulation; default: the record evaluated in fp64 and rounded once, the
              current raster.hip setup_kernel / setup_bwd_chain) -- its error is the tests' "fp32 floor";
  pair32      table fp64, per-pair fp32 (a GPU whose setup_bwd chain ran in fp64);
  table32     table fp32, per-pair fp64;
With the fp64 record (default) "table32" means the fp64 record rounded to fp32, so pair64/table32 isolates the
rounding of the stored record: exact arithmetic everywhere else -- the conditioning floor of an fp32 record.
  fp32+hp     the build: fp32, with the near-edge-on splats' (|normal . view| < 0.1) homogeneous point p evaluated from
              their fp64 record (raster.hip hit_p_hp; the oracle's RasterInputs.hp)
  hp<c        --hp-cos c: as pair64/table32, but the table of the near-edge-on splats (|normal . view| < c) kept fp64
Test infrastructure only (imports oracle/).  Usage: python tools/grad_precision.py [--win 48] [--cfg 3] [--hp-cos 0.05]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import DIFF, FLIP_MARGIN, grad_norm_err, grad_rel_err, make_case, make_window_case, upstream  # noqa: E402
from oracle import raster as O  # noqa: E402

F32, F64 = torch.float32, torch.float64


def grads(case, pair_dtype, table_dtype, outputs):
    inp = case.inp
    leaves = {}
    for k in DIFF:
        t = getattr(inp, k).detach().clone().requires_grad_(True)
        setattr(inp, k, t)
        leaves[k] = t
    _, o, aux = O.rasterize(inp, grad_dtype=pair_dtype, table_dtype=table_dtype)
    up = upstream(inp.cam.H, inp.cam.W, case.C, 5, aux["margin"] < FLIP_MARGIN)
    loss = sum((o[k] * up[k].to(pair_dtype)).sum() for k in outputs)
    loss.backward()
    out = {k: (v.grad.detach().double() if v.grad is not None else torch.zeros_like(v, dtype=F64)) for k, v in leaves.items()}
    for k in DIFF:
        setattr(inp, k, getattr(inp, k).detach())
    return out


GRAD32 = False  # --grad32: the table's gradient (the per-splat sums the GPU reduces and accumulates) rounded to fp32


def hp_mask_table(case, thr):
    """Precision analysis of raster.hip's near-edge-on path (GSTEX_HP_COS): in the gradient pass, the per-splat table of
    the splats with |normal . view direction| < thr stays fp64 while the others are rounded to fp32 -- what
    gstex_raster_setup_hp / gstex_raster_bwd_hp do (fp64 dx, dy, 1 / p.z, u, v for those splats).  Returns a restore
    function (patches the oracle; decisions stay the fp32 pass's)."""
    inp = case.inp
    with torch.no_grad():
        _, _, tw = O.quat_frame(inp.quats.double())
        _, cp, *_ = inp.cam.cast(F64)
        d = cp[None] - inp.means.double()
        mask = O._dot3(tw, d / d.norm(dim=-1, keepdim=True)).abs() < thr
    orig_table, orig_render = O._splat_table, O._render
    state = {"grad": False}

    def render(inp_, dtype, tr, si, decisions, edit=None, table_dtype=None):
        state["grad"] = table_dtype is not None
        try:
            return orig_render(inp_, dtype, tr, si, decisions, edit=edit, table_dtype=table_dtype)
        finally:
            state["grad"] = False

    def table(inp_, dtype):
        if dtype != F32 or not state["grad"]:
            return orig_table(inp_, dtype)
        t64 = orig_table(inp_, F64)
        if GRAD32:
            for v in t64.values():
                if v.is_floating_point() and v.requires_grad:
                    v.register_hook(lambda g: g.float().double())
        return {k: (torch.where(mask.view(-1, *([1] * (v.dim() - 1))), v, v.float().double()) if v.is_floating_point()
                    else v) for k, v in t64.items()}

    O._splat_table, O._render = table, render

    def restore():
        O._splat_table, O._render = orig_table, orig_render
    return float(mask.double().mean()), restore


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--win", type=int, default=48)
    ap.add_argument("--cfg", type=int, default=3)
    ap.add_argument("--all-outputs", action="store_true")
    ap.add_argument("--case", default=None,
                    help="a tests/test_gpu_parity.py CASES entry, or cfg1 (tests/test_gpu_deep.py), instead of a window")
    ap.add_argument("--fp32-record", action="store_true", help="all-fp32 per-splat record (round-2 formulation)")
    ap.add_argument("--hp-cos", type=float, nargs="*", default=[],
                    help="also: the table of splats with |normal . view dir| < each value kept fp64 (raster.hip GSTEX_HP_COS)")
    ap.add_argument("--grad32", action="store_true",
                    help="with --hp-cos: the per-splat table gradient rounded to fp32 (the GPU's fp32 sums)")
    ap.add_argument("--hp-sum32", action="store_true",
                    help="the fp32+hp row with the near-edge-on splats' p gradient summed in fp32 (as the HIP backward)")
    args = ap.parse_args()
    O.HP_SUM32 = args.hp_sum32
    global GRAD32
    GRAD32 = args.grad32
    O.RECORD_FP64 = not args.fp32_record
    outputs = ("img", "depth", "reg", "alpha", "tex", "normal") if args.all_outputs else ("img", "alpha", "tex")
    if args.case == "cfg1":
        case = make_case(n=1000, n_texels=0, H=256, W=256, seed=42, opacity=0.1)
    elif args.case:
        from test_gpu_parity import CASES
        case = make_case(**CASES[args.case])
    else:
        n, t = (200_000, 1e7) if args.cfg == 3 else (50_000, 1e6)
        case = make_window_case(n, t, 800, 800, args.win)
    case.inp.hp = False  # the historical mixes: no near-edge-on path (the "fp32+hp" row below is the build)
    ref = grads(case, F64, F64, outputs)
    mixes = {"fp32": (F32, F32), "pair32/table64": (F32, F64), "pair64/table32": (F64, F32)}
    print(f"{args.case or f'cfg{args.cfg} {args.win}x{args.win} window'}, {case.inp.means.shape[0]} splats, outputs {outputs}")
    print(f"{'mix':16s} " + " ".join(f"{k:>18s}" for k in DIFF))
    for name, (pd, td) in mixes.items():
        g = grads(case, pd, td, outputs)
        cells = []
        for k in DIFF:
            cells.append(f"{grad_norm_err(g[k], ref[k]):.2e}/{grad_rel_err(g[k], ref[k])[0]:.2e}")
        print(f"{name:16s} " + " ".join(f"{c:>18s}" for c in cells))
    # the build: fp32, with the near-edge-on splats' homogeneous point from their fp64 record (raster.hip hit_p_hp)
    case.inp.hp = True
    g = grads(case, F32, F32, outputs)
    frac = float(O._splat_table(case.inp, F64)["hp"].double().mean())
    cells = [f"{grad_norm_err(g[k], ref[k]):.2e}/{grad_rel_err(g[k], ref[k])[0]:.2e}" for k in DIFF]
    print(f"{'fp32+hp (' + f'{100 * frac:.1f}%)':16s} " + " ".join(f"{c:>18s}" for c in cells))
    case.inp.hp = False
    for thr in args.hp_cos:
        frac, restore = hp_mask_table(case, thr)
        g = grads(case, F64, F32, outputs)
        restore()
        cells = [f"{grad_norm_err(g[k], ref[k]):.2e}/{grad_rel_err(g[k], ref[k])[0]:.2e}" for k in DIFF]
        print(f"{'hp<' + str(thr) + f' ({100 * frac:.1f}%)':16s} " + " ".join(f"{c:>18s}" for c in cells))
    print("(norm-wise / max-element relative error vs all-fp64)")


if __name__ == "__main__":
    main()
