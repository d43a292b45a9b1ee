#!/usr/bin/env python3
"""CPU emulation of raster.hip's backward recurrences, to locate the means / quats error of the HIP backward on
near-edge-on splats (precision analysis, test infrastructure: imports oracle/).  The oracle's fp32 gradient pass
supplies every pair's fp32 values (u, v, 1/p.z, rho branch, depth, G, alpha, decisions) and every pixel's final state;
the emulation then walks each pixel's list back to front exactly as raster_bwd_kernel does (T recovered by division,
the colour behind R by recurrence, the distortion from the final M1 / M2), in fp32 or fp64, forms the per-pair
partials, sums them per splat in fp64 and pushes them through the fp64 record's autograd (the oracle's table).
Knobs (comma-separated, second argument): t64 (T and R recurrences in fp64), g64 (the per-pair gradient arithmetic in
fp64 from the fp32 pair values), s32 (per-splat sums rounded to fp32, as the GPU's accumulators), anch (the GPU's
anchored chain instead of the oracle table's autograd), acc32 (fp32 running sums, one fp32 partial per tile).
Usage: python tools/bwd_emulate.py [cfg1|no_reg|<CASES name>] [knobs]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import DIFF, make_case, oracle_run, upstream  # noqa: E402
from oracle import raster as O  # noqa: E402

F32, F64 = torch.float32, torch.float64


def make(name):
    if name == "cfg1":
        return make_case(n=1000, n_texels=0, H=256, W=256, seed=42, opacity=0.1)
    from test_gpu_parity import CASES
    return make_case(**CASES[name])


def emulate(case, knobs, flip_mask=None):
    """-> (per-splat sums dict (fp64), fp64 oracle gradients, leaves, fp64 table)"""
    _, _, aux, og = oracle_run(case, grads=True, flip_mask=flip_mask)
    inp = case.inp
    leaves = {}
    for k in DIFF:
        t = getattr(inp, k).detach().clone().requires_grad_(True)
        setattr(inp, k, t)
        leaves[k] = t
    O.CAPTURE = []
    with torch.no_grad():
        O.rasterize(inp, grad_dtype=F32)
    caps, O.CAPTURE = O.CAPTURE, None
    H, W = inp.cam.H, inp.cam.W
    up = upstream(H, W, case.C, 5, case.flip_mask)
    aa = bool(inp.settings & O.SETTING_AA_BLUR)
    dreg = bool(inp.settings & O.SETTING_DIST_REG)
    n = inp.means.shape[0]
    tdt = F64 if "t64" in knobs else F32
    gdt = F64 if "g64" in knobs else F32
    sums = {k: torch.zeros((n, d), dtype=F64) for k, d in
            (("A", 3), ("B", 3), ("P0", 3), ("TW", 3), ("XY", 2), ("OPAC", 1), ("RGB", 3), ("NRM", 3), ("XA", 1),
             ("YA", 1))}
    tab = O._splat_table(inp, F64)

    def add(key, gid, x):
        if "acc32" in knobs:  # fp32 running sums, one fp32 partial per tile (the GPU's wave reduce + float atomics)
            sums[key][gid] = (sums[key][gid].float() + x.float()).double()
        else:
            sums[key][gid] += x
    near, far = float(O.K_NEAR), float(O.K_FAR_RATIO)
    for rec in caps:
        if "u" not in rec:
            continue
        ids = rec["ids"]
        K = ids.numel()
        pix = torch.from_numpy(rec["pyi"] * W + rec["pxi"])
        px = torch.from_numpy(rec["pxi"]).float() + 0.5
        py = torch.from_numpy(rec["pyi"]).float() + 0.5
        Gimg = up["img"].reshape(-1, 3)[pix].to(gdt)
        Ga = up["alpha"].reshape(-1)[pix].to(gdt)
        Gd = up["depth"].reshape(-1)[pix].to(gdt)
        Greg = (up["reg"].reshape(-1)[pix] if dreg else torch.zeros(len(pix))).to(gdt)
        Gn = up["normal"].reshape(-1, 3)[pix].to(gdt)
        Gtex = up["tex"].reshape(-1, case.C)[pix].to(gdt)
        T = rec["Tfin"].to(tdt)
        Af = (1.0 - rec["Tfin"]).to(gdt)
        M1f, M2f = rec["M1"].to(gdt), rec["M2"].to(gdt)
        R = torch.zeros(len(pix), dtype=tdt)
        hp = rec["hp"]
        dxg = torch.where(hp[:, None], rec["dx64"].float(), rec["dx32"]).to(gdt)
        dyg = torch.where(hp[:, None], rec["dy64"].float(), rec["dy32"]).to(gdt)
        for j in range(K - 1, -1, -1):
            c = rec["incl"][j]
            if not bool(c.any()):
                continue
            a = rec["alpha"][j].to(tdt)
            one_m = 1.0 - a
            Tn = T / one_m
            T = torch.where(c, Tn, T)
            w = (a * T).to(gdt)
            u, v, ipz = rec["u"][j].to(gdt), rec["v"][j].to(gdt), rec["ipz"][j].to(gdt)
            z = rec["zz"][j].to(gdt)
            use3 = rec["use3"][j]
            rgb, nrm, Tw = rec["rgb"][j].to(gdt), rec["nrm"][j].to(gdt), rec["Tw"][j].to(gdt)
            g = (Gimg * rgb).sum(-1) + Gd * z + (Gn * nrm).sum(-1) + Ga
            dz = w * Gd
            if dreg:
                iz = 1.0 / z
                m = far * (1.0 - near * iz)
                E = (m * m * Af - 2.0 * m * M1f) + M2f
                g = g + Greg * E
                dz = dz + Greg * (2.0 * w * (m * Af - M1f)) * (far * near * iz * iz)
            # (texture: this emulation covers cases without texels -- their g and coordinate gradients are absent)
            dL = T.to(gdt) * (g - R.to(gdt))
            Rn = a * g.to(tdt) + one_m * R
            R = torch.where(c, Rn, R)
            ncl = ~rec["aclamp"][j]
            Gp = rec["G"][j].to(gdt)
            araw = rec["a_raw"][j].to(gdt)
            P_OPAC = torch.where(ncl, dL * Gp, torch.zeros_like(dL))
            drho = torch.where(ncl, dL * araw * -0.5, torch.zeros_like(dL))
            du = torch.where(use3, drho * 2.0 * u + dz * Tw[0], torch.zeros_like(dL))
            dv = torch.where(use3, drho * 2.0 * v + dz * Tw[1], torch.zeros_like(dL))
            xy = rec["xy"][j].to(gdt)
            P_XY = torch.stack([torch.where(use3, 0.0 * dL, drho * 4.0 * (xy[0] - px.to(gdt))),
                                torch.where(use3, 0.0 * dL, drho * 4.0 * (xy[1] - py.to(gdt)))], -1)
            dp = torch.stack([du * ipz, dv * ipz, -(du * u + dv * v) * ipz], -1)
            cm = c[:, None].to(gdt)
            dp = dp * cm
            gid = int(ids[j])
            add("A", gid, (dp * dxg[j][:, None]).double().sum(0))
            add("B", gid, (dp * dyg[j][:, None]).double().sum(0))
            add("P0", gid, dp.double().sum(0))
            tw3 = torch.stack([torch.where(use3, dz * u, 0 * dz), torch.where(use3, dz * v, 0 * dz), dz], -1)
            add("TW", gid, (tw3 * cm).double().sum(0))
            add("XY", gid, (P_XY * cm).double().sum(0))
            add("OPAC", gid, (P_OPAC * c.to(gdt)).double().sum())
            add("RGB", gid, ((w[:, None] * Gimg) * cm).double().sum(0))
            add("NRM", gid, ((w[:, None] * Gn) * cm).double().sum(0))
    return sums, og, leaves, tab


def chain(case, sums, leaves, tab, knobs):
    """The per-splat sums through the fp64 record chain -> dict of leaf gradients (+ centers)."""
    inp = case.inp
    n = inp.means.shape[0]
    sums = dict(sums)
    sums.setdefault("XA", torch.zeros((n, 1), dtype=F64))
    sums.setdefault("YA", torch.zeros((n, 1), dtype=F64))
    if "s32" in knobs:  # the GPU's per-splat sums are fp32
        sums = {k: v.float().double() for k, v in sums.items()}
    if "anch" in knobs:
        # raster.hip setup_bwd_chain: the anchored vjp (anchor held fixed, the zero-valued z components of Tu', Tv'
        # carry gradient), fp64
        V, campos, fx, fy, cx, cy = inp.cam.cast(F64)
        tu, tv, tw = O.quat_frame(leaves["quats"].to(F64))
        su = leaves["scales"][:, 0].to(F64) * float(inp.glob_scale)
        sv = leaves["scales"][:, 1].to(F64) * float(inp.glob_scale)
        a, b, mu = tu * su[:, None], tv * sv[:, None], leaves["means"].to(F64)
        W0 = [O._vrow(V, r, a) for r in range(3)]
        W1 = [O._vrow(V, r, b) for r in range(3)]
        W2 = [O._vrow(V, r, mu) + V[r, 3] for r in range(3)]
        xn = (W2[0] / W2[2]).detach()
        yn = (W2[1] / W2[2]).detach()
        Tu = torch.stack([fx * (W0[0] - xn * W0[2]), fx * (W1[0] - xn * W1[2]), fx * (W2[0] - xn * W2[2])], -1)
        Tv = torch.stack([fy * (W0[1] - yn * W0[2]), fy * (W1[1] - yn * W1[2]), fy * (W2[1] - yn * W2[2])], -1)
        Tw = torch.stack([W0[2], W1[2], W2[2]], -1)
        Aa, Ba, P0a = torch.cross(Tv, Tw, dim=-1), torch.cross(Tw, Tu, dim=-1), torch.cross(Tu, Tv, dim=-1)
        outs = [Aa, Ba, P0a, Tw, tab["opac"], tab["rgb"], tab["nrm"]]
        gos = [sums["A"], sums["B"], sums["P0"], sums["TW"], sums["OPAC"][:, 0], sums["RGB"], sums["NRM"]]
    else:
        # the anchor path of the oracle's table (dx = px - xa): -sum dp . A, -sum dp . B
        A, B = tab["A"].detach(), tab["B"].detach()
        sums["XA"][:, 0] = -(sums["P0"] * A).sum(-1)
        sums["YA"][:, 0] = -(sums["P0"] * B).sum(-1)
        outs = [tab["A"], tab["B"], tab["Pz"], tab["Tw"], tab["opac"], tab["rgb"], tab["nrm"], tab["xa"], tab["ya"]]
        gos = [sums["A"], sums["B"], sums["P0"][:, 2], sums["TW"], sums["OPAC"][:, 0], sums["RGB"], sums["NRM"],
               sums["XA"][:, 0], sums["YA"][:, 0]]
    gr = torch.autograd.grad(outs, [leaves[k] for k in ("means", "quats", "scales", "opacities", "rgbs")],
                             grad_outputs=gos, allow_unused=True, retain_graph=True)
    out = dict(zip(("means", "quats", "scales", "opacities", "rgbs"), gr))
    out["centers"] = sums["XY"]
    return out


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg1"
    knobs = set(sys.argv[2].split(",")) if len(sys.argv) > 2 else set()
    case = make(name)
    sums, og, leaves, tab = emulate(case, knobs)
    gr = chain(case, sums, leaves, tab, knobs)
    print(f"{name} knobs={sorted(knobs)}: emulated backward vs fp64 oracle (norm-wise relative)")
    for k, gk in gr.items():
        ref = og[k].double()
        print(f"  {k:10s} {float((gk - ref).norm() / ref.norm()):.3e}")


if __name__ == "__main__":
    main()
