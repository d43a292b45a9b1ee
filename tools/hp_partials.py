#!/usr/bin/env python3
"""Per-splat backward sums, GPU vs the CPU emulation of the same recurrences (precision analysis of the near-edge-on
path, test infrastructure).
  gpu CASE OUT.pt : (GPU box) run the HIP raster forward / backward of the parity case, keep the per-splat float-atomic
                    sums (ops.PARTIALS_HOOK) and the leaf gradients
  cpu CASE OUT.pt : compare them with tools/bwd_emulate.py's sums (field by field, near-edge-on splats apart) and push
                    the GPU's sums through the emulation's fp64 chain (does the chain reproduce the GPU's gradients?)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from helpers import gpu_run, oracle_run  # noqa: E402
import bwd_emulate as E  # noqa: E402

FIELDS = dict(A=(0, 3), B=(3, 3), P0=(6, 3), XY=(9, 2), OPAC=(11, 1), RGB=(12, 3), NRM=(21, 3), TW=(24, 3))


def main():
    mode, name, path = sys.argv[1], sys.argv[2], sys.argv[3]
    case = E.make(name)
    if mode == "gpu":
        from gstex_amd import ops
        oracle_run(case, grads=False)  # the flip mask the upstream gradient uses
        got = []
        ops.PARTIALS_HOOK = lambda p, f, r, h: got.append((p.detach().clone().cpu(), r.detach().clone().cpu(),
                                                            None if h is None else h.detach().clone().cpu()))
        _, gr = gpu_run(case, grads=True)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        torch.save({"partials": got[0][0], "records": got[0][1], "hp": got[0][2], "grads": gr,
                    "flip_mask": case.flip_mask}, path)
        print(f"saved {tuple(got[0][0].shape)} partials to {path}")
        return
    d = torch.load(path, weights_only=True)
    P = d["partials"].double()
    sums, og, leaves, tab = E.emulate(case, set(), flip_mask=d.get("flip_mask"))
    hp = tab["hp"]
    print(f"{name}: {int(hp.sum())} near-edge-on splats of {hp.numel()}")
    gsum = {}
    for k, (o, w) in FIELDS.items():
        if P.shape[1] < o + w:
            continue
        g = P[:, o:o + w]
        gsum[k] = g
        e = sums[k]
        for lab, m in (("hp", hp), ("rest", ~hp)):
            ref = e[m]
            err = (g[m] - ref).norm() / ref.norm().clamp_min(1e-30)
            print(f"  {k:5s} {lab:4s} GPU vs emulated sums: {float(err):.3e}")
    for k in ("A", "B", "P0", "XY", "OPAC", "RGB", "NRM", "TW"):
        gsum.setdefault(k, torch.zeros_like(sums[k]))
    for lab, s in (("emulated sums", sums), ("GPU sums", gsum)):
        gr = E.chain(case, s, leaves, tab, {"anch"})
        print(f"  chain({lab}) vs fp64 oracle / vs GPU gradients:")
        for k, gk in gr.items():
            ref = og[k].double()
            gg = d["grads"][k].double()
            print(f"    {k:10s} {float((gk - ref).norm() / ref.norm()):.3e} / {float((gk - gg).norm() / gg.norm()):.3e}")
    print("  GPU gradients vs fp64 oracle:")
    for k in ("means", "quats", "scales", "opacities", "rgbs", "centers"):
        ref = og[k].double()
        print(f"    {k:10s} {float((d['grads'][k].double() - ref).norm() / ref.norm()):.3e}")


if __name__ == "__main__":
    main()
