#!/usr/bin/env python3
"""Where does the HIP backward's remaining means / quats error sit?  (Diagnostic, test infrastructure: imports oracle/.)
For a parity case: the HIP gradients in the atomic (default) and the deterministic (per-pair rows, fixed-order sums)
modes against the fp64 oracle; the splats with the largest means / quats error, whether they are near edge-on
(|normal . view| < 0.1, the hp mark), their |cos| and their tile-pair counts.
Usage (GPU box): python tools/hp_diag.py [cfg1|cfg3w|<CASES name>]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import DIFF, gpu_run, grad_norm_err, make_case, make_window_case, oracle_run  # noqa: E402
from oracle import raster as O  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg1"
    outputs = None
    if name == "cfg1":
        case = make_case(n=1000, n_texels=0, H=256, W=256, seed=42, opacity=0.1)
    elif name == "cfg3w":
        case = make_window_case(200_000, 1e7, 800, 800, 96)
        outputs = ("img", "alpha", "tex")
    else:
        from test_gpu_parity import CASES
        case = make_case(**CASES[name])
    _, _, aux, og = oracle_run(case, grads=True, outputs=outputs)
    _, _, _, og32 = oracle_run(case, grads=True, grad_dtype=torch.float32, outputs=outputs)
    _, gg = gpu_run(case, grads=True, outputs=outputs)
    torch.use_deterministic_algorithms(True)
    try:
        _, gd = gpu_run(case, grads=True, outputs=outputs)
    finally:
        torch.use_deterministic_algorithms(False)
    for k in DIFF:
        print(f"{k:10s} atomic {grad_norm_err(gg[k], og[k]):.2e}  rows {grad_norm_err(gd[k], og[k]):.2e}  "
              f"oracle fp32 {grad_norm_err(og32[k], og[k]):.2e}  atomic-vs-rows {grad_norm_err(gg[k], gd[k]):.2e}")
    inp = case.inp
    with torch.no_grad():
        _, _, tw = O.quat_frame(inp.quats.double())
        _, cp, *_ = inp.cam.cast(torch.float64)
        d = cp[None] - inp.means.double()
        cos = (O._dot3(tw, d) / d.norm(dim=-1)).abs()
    nth = case.nth
    for k in ("means", "quats"):
        e = (gg[k].double() - og[k].double()).norm(dim=-1)
        tot = float((og[k].double().norm(dim=-1) ** 2).sum().sqrt())
        top = torch.argsort(e, descending=True)[:12]
        share = float((e[top] ** 2).sum() / (e ** 2).sum())
        print(f"{k}: |err| total {float(e.norm()):.3e} of |grad| {tot:.3e}; top-12 splats carry {100 * share:.0f}% "
              f"of the squared error")
        for g in top.tolist():
            print(f"   splat {g:6d} err {float(e[g]):.3e} |grad| {float(og[k][g].double().norm()):.3e} "
                  f"rows-err {float((gd[k][g].double() - og[k][g].double()).norm()):.3e} |cos| {float(cos[g]):.4f} "
                  f"hp {bool(cos[g] < O.K_HP_COS)} tiles {int(nth[g])} opac {float(inp.opacities[g]):.3f}")


if __name__ == "__main__":
    main()
