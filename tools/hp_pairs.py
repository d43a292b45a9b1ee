#!/usr/bin/env python3
"""Per-pair backward values, GPU vs the oracle's fp32 pass (precision analysis, test infrastructure).
  gpu CASE OUT.pt [GID...] : (GPU box, GSTEX_LIB=scratch/pairs/libgstex_hip.so from tools/build_variant.sh pairs
                    -DGSTEX_PAIR_DUMP) the HIP backward of the parity case, the contributing pairs of the
                    near-edge-on splats and of the splats GID...
  cpu CASE OUT.pt : match the records to the oracle's captured pairs (gid, pixel) and report the largest relative
                    differences per field, near-edge-on splats apart, plus pairs present on one side only"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from helpers import gpu_run, oracle_run, upstream  # noqa: E402
import bwd_emulate as E  # noqa: E402
from oracle import raster as O  # noqa: E402

NAMES = ["gid", "px", "py", "flags", "T", "w", "dL", "drho", "u", "v", "ipz", "z", "alpha", "G", "dx", "dy"]


def main():
    mode, name, path = sys.argv[1], sys.argv[2], sys.argv[3]
    case = E.make(name)
    if mode == "gpu":
        from gstex_amd import _lib
        lib = _lib.load()
        oracle_run(case, grads=False)
        cap = 4 << 20
        buf = torch.zeros((cap, 16), device="cuda", dtype=torch.float32)
        cnt = torch.zeros((1,), device="cuda", dtype=torch.int32)
        torch.cuda.synchronize()
        assert lib.gstex_debug_pair_dump(ctypes.c_void_p(buf.data_ptr()), ctypes.c_int(cap),
                                         ctypes.c_void_p(cnt.data_ptr())) == 0
        gpu_run(case, grads=True)
        torch.cuda.synchronize()
        n = int(cnt.item())
        lib.gstex_debug_pair_dump(None, 0, None)
        assert n <= cap, n
        rec = buf[:n].cpu()
        # keep the near-edge-on splats' pairs and those of the splats named on the command line (the output must stay
        # small enough to travel back)
        keep = O._splat_table(case.inp, torch.float64)["hp"].clone()
        for a in sys.argv[4:]:
            keep[int(a)] = True
        rec = rec[keep[rec[:, 0].view(torch.int32).long()]]
        torch.save({"pairs": rec}, path)
        print(f"saved {rec.shape[0]} of {n} pair records to {path}")
        return
    rec = torch.load(path, weights_only=True)["pairs"]
    gid = rec[:, 0].view(torch.int32).long()
    flags = rec[:, 3].view(torch.int32)
    pix_g = (rec[:, 2].floor().long() * case.inp.cam.W + rec[:, 1].floor().long())
    kept = set(gid.unique().tolist())
    # oracle side
    inp = case.inp
    oracle_run(case, grads=False)
    O.CAPTURE = []
    with torch.no_grad():
        O.rasterize(inp, grad_dtype=torch.float32)
    caps, O.CAPTURE = O.CAPTURE, None
    W = inp.cam.W
    tab = O._splat_table(inp, torch.float64)
    hp = tab["hp"]
    ok_ids, ok_pix, vals = [], [], {k: [] for k in ("u", "v", "ipz", "zz", "alpha", "G", "use3", "aclamp")}
    for c in caps:
        if "u" not in c:
            continue
        inc = c["incl"]
        kk, pp = torch.nonzero(inc, as_tuple=True)
        ok_ids.append(c["ids"][kk].long())
        pix = torch.from_numpy(c["pyi"] * W + c["pxi"]).long()
        ok_pix.append(pix[pp])
        for k in vals:
            vals[k].append(c[k][kk, pp])
    oid = torch.cat(ok_ids)
    sel = torch.isin(oid, torch.tensor(sorted(kept)))
    oid = oid[sel]
    opix = torch.cat(ok_pix)[sel]
    ov = {k: torch.cat(v)[sel] for k, v in vals.items()}
    key_o = oid * (1 << 24) + opix
    key_g = gid * (1 << 24) + pix_g
    print(f"{name}: GPU {len(key_g)} contributing pairs, oracle {len(key_o)}")
    so, io = torch.sort(key_o)
    sg, ig = torch.sort(key_g)
    only_g = ~torch.isin(sg, so)
    only_o = ~torch.isin(so, sg)
    print(f"  pairs only on the GPU: {int(only_g.sum())}, only in the oracle: {int(only_o.sum())}")
    for lab, keys in (("GPU-only", sg[only_g][:10]), ("oracle-only", so[only_o][:10])):
        for k in keys.tolist():
            print(f"    {lab}: splat {k >> 24} (hp={bool(hp[k >> 24])}) pixel {k & ((1 << 24) - 1)}")
    common = torch.isin(sg, so)
    gi = ig[common]
    pos = torch.searchsorted(so, sg[common])
    oi = io[pos]
    use3_g = (flags[gi] & 1) != 0
    use3_o = ov["use3"][oi]
    flip = use3_g != use3_o
    print(f"  use3 branch differs on {int(flip.sum())} common pairs")
    for i in torch.nonzero(flip)[:10, 0].tolist():
        g, o = gi[i], oi[i]
        print(f"    splat {int(gid[g])} (hp={bool(hp[gid[g]])}) pixel {int(pix_g[g])}: GPU use3={bool(use3_g[i])} "
              f"u {float(rec[g, 8]):.9g} v {float(rec[g, 9]):.9g} | oracle u {float(ov['u'][o]):.9g} v {float(ov['v'][o]):.9g}")
    for fname, col, okey in (("u", 8, "u"), ("v", 9, "v"), ("ipz", 10, "ipz"), ("z", 11, "zz"), ("alpha", 12, "alpha"),
                             ("G", 13, "G")):
        a = rec[gi, col].double()
        b = ov[okey][oi].double()
        rel = (a - b).abs() / b.abs().clamp_min(1e-30)
        for lab, m in (("hp", hp[gid[gi]]), ("rest", ~hp[gid[gi]])):
            r = rel[m & ~flip]
            if r.numel():
                j = int(torch.argmax(r))
                print(f"  {fname:5s} {lab:4s} rel diff max {float(r.max()):.3e} median {float(r.median()):.3e}")


if __name__ == "__main__":
    main()
