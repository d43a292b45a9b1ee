#!/usr/bin/env python3
"""How much of the HIP backward's means / quats error does the precision of the dL/d(A, B, Pz) sums explain?
(Precision analysis, test infrastructure: imports oracle/.)  The oracle's fp32 gradient pass (with the near-edge-on p
from the fp64 record, as the HIP kernels) hands over every pair's dL/dp; the per-splat sums dL/dA = sum dp dx,
dL/dB = sum dp dy, dL/dPz = sum dp.z are then formed
  exact   in fp64 with the fp64 offsets,
  gpu     as raster.hip does: fp32 products, fp32 sums per 8x8 quadrant (one backward visit), fp32 accumulation of the
          visits (the per-splat float atomics),
  and the variants named on the command line,
and each is pushed through the same fp64 chain (autograd of the fp64 record); the printed error is relative to the
norm of the exact fp64 gradient of means / quats.
Usage: python tools/hp_sum_model.py [cfg1|cfg3w|<CASES name>]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import DIFF, make_case, make_window_case, oracle_run, upstream  # noqa: E402
from oracle import raster as O  # noqa: E402

F32, F64 = torch.float32, torch.float64


def build(name):
    if name == "cfg1":
        return make_case(n=1000, n_texels=0, H=256, W=256, seed=42, opacity=0.1), None
    if name == "cfg3w":
        return make_window_case(200_000, 1e7, 800, 800, 96), ("img", "alpha", "tex")
    from test_gpu_parity import CASES
    return make_case(**CASES[name]), None


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg1"
    case, outputs = build(name)
    _, _, aux, og = oracle_run(case, grads=True, outputs=outputs)  # fp64 reference (and case.flip_mask)
    inp = case.inp
    leaves = {}
    for k in DIFF:
        t = getattr(inp, k).detach().clone().requires_grad_(True)
        setattr(inp, k, t)
        leaves[k] = t
    O.CAPTURE = []
    _, o, _ = O.rasterize(inp, grad_dtype=F32)
    up = upstream(inp.cam.H, inp.cam.W, case.C, 5, case.flip_mask)
    names = outputs or ("img", "depth", "reg", "alpha", "tex", "normal")
    if inp.settings & O.SETTING_EVAL_NORMAL:
        names = tuple(k for k in names if k != "normal")
    loss = sum((o[k] * up[k].to(F32)).sum() for k in names)
    loss.backward()
    caps, O.CAPTURE = O.CAPTURE, None
    n = inp.means.shape[0]
    W = inp.cam.W

    def sums(mode):
        acc = {k: torch.zeros((n, 3), dtype=F64 if mode != "gpu" else F32) for k in ("A", "B")}
        acc["P"] = torch.zeros((n, 3), dtype=F64 if mode != "gpu" else F32)
        for rec in caps:
            if "gx" not in rec:
                continue
            gp = torch.stack([rec["gx"], rec["gy"], rec["gz"]], -1)  # (K, P, 3) fp32
            ids = rec["ids"]
            if mode == "exact":
                dx, dy = rec["dx64"], rec["dy64"]
                acc["A"].index_add_(0, ids, (gp.double() * dx[..., None]).sum(1))
                acc["B"].index_add_(0, ids, (gp.double() * dy[..., None]).sum(1))
                acc["P"].index_add_(0, ids, gp.double().sum(1))
                continue
            # per 8x8 quadrant of the tile: the backward's visit
            q = torch.from_numpy(((rec["pyi"] // 8) % 2) * 2 + ((rec["pxi"] // 8) % 2))
            dx = rec["dx64"].float()
            dy = rec["dy64"].float()
            for qq in range(4):
                m = q == qq
                if not bool(m.any()):
                    continue
                g = gp[:, m]
                if mode == "gpu":
                    sA = (g * dx[:, m, None]).sum(1)  # fp32 products and sums
                    sB = (g * dy[:, m, None]).sum(1)
                    sP = g.sum(1)
                    for key, v in (("A", sA), ("B", sB), ("P", sP)):
                        acc[key].index_add_(0, ids, v)  # fp32 accumulation
                elif mode == "centered":  # offsets from the quadrant centre in fp32, the anchor term added in fp64
                    cx = float(rec["pxi"][m.numpy()].mean()) + 0.5
                    cy = float(rec["pyi"][m.numpy()].mean()) + 0.5
                    d0x = rec["dx64"][:, m][:, :1] - (torch.from_numpy(rec["pxi"][m.numpy()][:1].astype(np.float64)) + 0.5 - cx)
                    d0y = rec["dy64"][:, m][:, :1] - (torch.from_numpy(rec["pyi"][m.numpy()][:1].astype(np.float64)) + 0.5 - cy)
                    ox = (torch.from_numpy(rec["pxi"][m.numpy()].astype(np.float32)) + 0.5 - cx)[None, :]
                    oy = (torch.from_numpy(rec["pyi"][m.numpy()].astype(np.float32)) + 0.5 - cy)[None, :]
                    sP = g.sum(1)
                    sA = (g * ox[..., None]).sum(1).double() + d0x * sP.double()
                    sB = (g * oy[..., None]).sum(1).double() + d0y * sP.double()
                    for key, v in (("A", sA), ("B", sB), ("P", sP.double())):
                        acc[key].index_add_(0, ids, v)
                elif mode == "fp64acc":  # fp32 products and quadrant sums, fp64 accumulation of the visits
                    sA = (g * dx[:, m, None]).sum(1)
                    sB = (g * dy[:, m, None]).sum(1)
                    sP = g.sum(1)
                    for key, v in (("A", sA), ("B", sB), ("P", sP)):
                        acc[key].index_add_(0, ids, v.double())
        return {k: v.double() for k, v in acc.items()}

    tab = O._splat_table(inp, F64)
    ref = {k: og[k].double() for k in ("means", "quats", "scales")}

    def chain(s):
        gr = torch.autograd.grad([tab["A"], tab["B"], tab["Pz"]], [leaves["means"], leaves["quats"], leaves["scales"]],
                                 grad_outputs=[s["A"], s["B"], s["P"][:, 2]], retain_graph=True, allow_unused=True)
        return dict(zip(("means", "quats", "scales"), gr))

    ex = chain(sums("exact"))
    print(f"{name}: relative to |exact fp64 gradient| (norm-wise)")
    for mode in ("gpu", "fp64acc", "centered"):
        gm = chain(sums(mode))
        cells = [f"{k} {float((gm[k] - ex[k]).norm() / ref[k].norm()):.2e}" for k in ("means", "quats", "scales")]
        print(f"  {mode:10s} " + "  ".join(cells))


if __name__ == "__main__":
    main()
