"""An independent statement of the forward the oracle restates (CPU, test infrastructure).

oracle/raster.py follows the kernels' own formulation (gstex_common.h: the anchored homography in affine form, p = dx A
+ dy B + (0, 0, Pz), u = p.x / p.z, ...), so agreeing with it alone does not show that formulation renders 2DGS
splats.  This file restates the forward from the 2DGS definitions instead, in float64 numpy: per pixel the camera ray
through the pixel centre, its intersection with each splat's plane in the splat's own frame (solving
c + u a + v b = lambda d, a = R t_u s_u, b = R t_v s_v in camera coordinates), rho3 = u^2 + v^2 against the screen-space
low-pass rho2 = 2 |centre - pixel|^2 (AA bit 9), alpha = min(0.99, o exp(-rho / 2)) with the 1/255 and near-plane
skips, front-to-back compositing in each tile's (depth, id) order with the T < 1e-4 termination, the hit point's
view depth, the camera-facing world normal, and the texel lookup at uv0 + (umap, vmap) . (hit - mu) in texel units
(corner-aligned bilinear, clamped to the block).  The per-tile lists are the oracle's binning (itself checked against
brute force in test_oracle.py).  Pixels whose oracle decisions lie within FLIP_MARGIN of a threshold are left out
(the oracle takes fp32 decisions, this restatement fp64 ones)."""
import numpy as np
import pytest
import torch

from helpers import FLIP_MARGIN, make_case
from oracle import raster as O

NEAR, AMAX, AMIN, TMIN = 0.2, 0.99, 1.0 / 255.0, 1e-4


def rotation(q):
    w, x, y, z = (q / np.linalg.norm(q, axis=-1, keepdims=True)).T
    return np.stack([np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)], -1),
                     np.stack([2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)], -1),
                     np.stack([2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1)], -2)


def ray_render(inp):
    cam = inp.cam
    H, W = cam.H, cam.W
    f32 = lambda v: float(np.float32(v))  # noqa: E731  (the kernels' float arguments)
    fx, fy, cx, cy = f32(cam.fx), f32(cam.fy), f32(cam.cx), f32(cam.cy)
    V = cam.viewmat.double().numpy()
    Rv, tv_ = V[:, :3], V[:, 3]
    campos = cam.campos.double().numpy()
    mu = inp.means.double().numpy()
    glob = f32(inp.glob_scale)
    su = inp.scales[:, 0].double().numpy() * glob
    sv = inp.scales[:, 1].double().numpy() * glob
    Rq = rotation(inp.quats.double().numpy())
    t_u, t_v, t_w = Rq[:, :, 0], Rq[:, :, 1], Rq[:, :, 2]
    c = mu @ Rv.T + tv_  # splat centres, camera coordinates
    a = (t_u * su[:, None]) @ Rv.T
    b = (t_v * sv[:, None]) @ Rv.T
    nrm = np.where((np.einsum("ij,ij->i", t_w, campos[None] - mu) < 0)[:, None], -t_w, t_w)
    opac = inp.opacities[:, 0].double().numpy()
    rgb = inp.rgbs.double().numpy()
    ctr = inp.centers.double().numpy()
    dims = inp.texture_dims.numpy().astype(np.int64)
    tex = inp.texture.double().numpy()
    uv0 = inp.uv0[:, 0, :].double().numpy()
    um, vm = inp.umap[:, 0, :].double().numpy(), inp.vmap[:, 0, :].double().numpy()
    aa = bool(inp.settings & O.SETTING_AA_BLUR)
    C = tex.shape[1]
    _, tile_ranges, sorted_ids, _ = O.bin_and_sort(inp.centers, inp.extents, inp.depths, H, W)
    tiles_x = (W + 15) // 16
    out = {k: np.zeros((H, W) + s) for k, s in (("img", (3,)), ("alpha", ()), ("depth", ()), ("tex", (C,)),
                                                  ("normal", (3,)))}
    for t, (s, e) in enumerate(tile_ranges):
        ids = sorted_ids[s:e]
        ty, tx = divmod(t, tiles_x)
        for py in range(ty * 16, min(ty * 16 + 16, H)):
            for px in range(tx * 16, min(tx * 16 + 16, W)):
                d = np.array([(px + 0.5 - cx) / fx, (py + 0.5 - cy) / fy, 1.0])
                T = 1.0
                acc = {k: np.zeros_like(v[0, 0]) for k, v in out.items()}
                for g in ids:
                    M = np.stack([a[g], b[g], -d], 1)
                    if abs(np.linalg.det(M)) < 1e-300:
                        continue
                    u, v, lam = np.linalg.solve(M, -c[g])
                    rho3 = u * u + v * v
                    rho2 = 2.0 * ((ctr[g, 0] - (px + 0.5)) ** 2 + (ctr[g, 1] - (py + 0.5)) ** 2)
                    use3 = (rho3 <= rho2) if aa else True
                    rho = rho3 if use3 else rho2
                    z = lam if use3 else c[g, 2]
                    alpha = min(AMAX, opac[g] * np.exp(-0.5 * rho))
                    if z < NEAR or alpha < AMIN:
                        continue
                    if T * (1.0 - alpha) < TMIN:
                        break
                    w = alpha * T
                    acc["img"] += w * rgb[g]
                    acc["depth"] += w * z
                    acc["normal"] += w * nrm[g]
                    h_, w_, off = dims[g]
                    if h_ * w_ > 0:
                        hit = mu[g] + u * su[g] * t_u[g] + v * sv[g] * t_v[g]
                        xr = h_ * (uv0[g, 0] + um[g] @ (hit - mu[g]))
                        yr = w_ * (uv0[g, 1] + vm[g] @ (hit - mu[g]))
                        x, y = min(max(xr, 0.0), h_ - 1.0), min(max(yr, 0.0), w_ - 1.0)
                        i0, j0 = int(x), int(y)
                        i1, j1 = min(i0 + 1, h_ - 1), min(j0 + 1, w_ - 1)
                        ax, ay = x - i0, y - j0
                        tx_ = lambda i, j: tex[off + i * w_ + j]  # noqa: E731
                        val = (1 - ax) * ((1 - ay) * tx_(i0, j0) + ay * tx_(i0, j1)) + \
                            ax * ((1 - ay) * tx_(i1, j0) + ay * tx_(i1, j1))
                        acc["tex"] += w * val
                    T *= 1.0 - alpha
                acc["alpha"] = 1.0 - T
                for k in out:
                    out[k][py, px] = acc[k]
    return out


@pytest.mark.parametrize("name,kw", [
    ("aa_dist", dict(n=120, n_texels=6000, H=40, W=48, seed=3)),
    ("no_aa", dict(n=120, n_texels=6000, H=40, W=48, seed=4, settings=1 << 10)),
    ("2dgs", dict(n=150, n_texels=0, H=32, W=48, seed=5)),
])
def test_world_space_ray_restatement_matches_oracle(name, kw):
    case = make_case(**kw)
    o32, o64, aux = O.rasterize(case.inp)
    ref = ray_render(case.inp)
    ok = (aux["margin"] >= FLIP_MARGIN).numpy()
    assert ok.mean() > 0.95
    assert float(ref["alpha"][ok].max()) > 0.5, "the scene must cover the image"
    for k in ("img", "alpha", "depth", "tex", "normal"):
        a = o64[k].double().numpy()[ok]
        b = ref[k][ok]
        err = float(np.abs(a - b).max())
        # fp64 both: agreement to rounding (the fp32 oracle output differs by ~2e-7 here, so this is a sharp check)
        assert err <= 1e-12 * max(1.0, float(np.abs(b).max())), f"{name}: {k} differs by {err:.3e}"


def ray_render_torch(inp, leaves):
    """The same world-space restatement in torch float64, differentiable w.r.t. the leaves (means, scales, quats,
    opacities, rgbs, texture, centers): per tile, every (splat, pixel) pair's ray-plane system solved by Cramer's
    rule, the pair decisions (skips, low-pass branch, termination) taken in float64 without gradient, the composite
    as a product scan.  Outputs img, alpha, depth, tex, normal of the whole image."""
    cam = inp.cam
    H, W = cam.H, cam.W
    f32 = lambda v: float(np.float32(v))  # noqa: E731
    fx, fy, cx, cy = f32(cam.fx), f32(cam.fy), f32(cam.cx), f32(cam.cy)
    F = torch.float64
    V = cam.viewmat.to(F)
    campos = cam.campos.to(F)
    mu = leaves["means"].to(F)
    glob = f32(inp.glob_scale)
    su = leaves["scales"][:, 0].to(F) * glob
    sv = leaves["scales"][:, 1].to(F) * glob
    q = leaves["quats"].to(F)
    q = q / q.norm(dim=-1, keepdim=True)
    w_, x_, y_, z_ = q.unbind(-1)
    t_u = torch.stack([1 - 2 * (y_ * y_ + z_ * z_), 2 * (x_ * y_ + w_ * z_), 2 * (x_ * z_ - w_ * y_)], -1)
    t_v = torch.stack([2 * (x_ * y_ - w_ * z_), 1 - 2 * (x_ * x_ + z_ * z_), 2 * (y_ * z_ + w_ * x_)], -1)
    t_w = torch.stack([2 * (x_ * z_ + w_ * y_), 2 * (y_ * z_ - w_ * x_), 1 - 2 * (x_ * x_ + y_ * y_)], -1)
    R, tt = V[:, :3], V[:, 3]
    c = mu @ R.T + tt
    a = (t_u * su[:, None]) @ R.T
    b = (t_v * sv[:, None]) @ R.T
    flip = ((t_w * (campos[None] - mu)).sum(-1) < 0).detach()
    nrm = torch.where(flip[:, None], -t_w, t_w)
    opac = leaves["opacities"][:, 0].to(F)
    rgb = leaves["rgbs"].to(F)
    ctr = leaves["centers"].to(F)
    tex = leaves["texture"].to(F)
    dims = inp.texture_dims.long()
    uv0 = inp.uv0[:, 0, :].to(F)
    um, vm = inp.umap[:, 0, :].to(F), inp.vmap[:, 0, :].to(F)
    aa = bool(inp.settings & O.SETTING_AA_BLUR)
    C = tex.shape[1]
    _, tile_ranges, sorted_ids, _ = O.bin_and_sort(inp.centers, inp.extents, inp.depths, H, W)
    tiles_x = (W + 15) // 16
    out = {k: torch.zeros((H, W) + s, dtype=F) for k, s in (("img", (3,)), ("alpha", ()), ("depth", ()),
                                                              ("tex", (C,)), ("normal", (3,)))}
    rows = {k: [] for k in out}
    pix_all = []
    for t, (s, e) in enumerate(tile_ranges):
        if e <= s:
            continue
        ids = torch.from_numpy(np.asarray(sorted_ids[s:e], dtype=np.int64))
        ty, tx = divmod(t, tiles_x)
        ys, xs = torch.meshgrid(torch.arange(ty * 16, min(ty * 16 + 16, H)), torch.arange(tx * 16, min(tx * 16 + 16, W)),
                                indexing="ij")
        ys, xs = ys.reshape(-1), xs.reshape(-1)
        d = torch.stack([(xs.to(F) + 0.5 - cx) / fx, (ys.to(F) + 0.5 - cy) / fy, torch.ones(len(xs), dtype=F)], -1)
        A_, B_, C_ = a[ids][:, None, :], b[ids][:, None, :], c[ids][:, None, :]
        D_ = -d[None, :, :]
        det = lambda p, q_, r: (p * torch.cross(q_, r, dim=-1)).sum(-1)  # noqa: E731
        M0 = det(A_.expand(-1, len(xs), -1), B_.expand(-1, len(xs), -1), D_.expand(len(ids), -1, -1))
        rhs = -C_.expand(-1, len(xs), -1)
        Ae, Be, De = A_.expand_as(rhs), B_.expand_as(rhs), D_.expand_as(rhs)
        u = det(rhs, Be, De) / M0
        v = det(Ae, rhs, De) / M0
        lam = det(Ae, Be, rhs) / M0
        rho3 = u * u + v * v
        rho2 = 2.0 * ((ctr[ids][:, None, 0] - (xs.to(F) + 0.5)[None]) ** 2 + (ctr[ids][:, None, 1] - (ys.to(F) + 0.5)[None]) ** 2)
        use3 = (rho3 <= rho2).detach() if aa else torch.ones_like(rho3, dtype=torch.bool)
        rho = torch.where(use3, rho3, rho2)
        z = torch.where(use3, lam, c[ids][:, None, 2].expand_as(lam))
        a_raw = opac[ids][:, None] * torch.exp(-0.5 * rho)
        alpha = torch.clamp(a_raw, max=AMAX)
        with torch.no_grad():
            valid = (z >= NEAR) & (alpha >= AMIN)
            ae = torch.where(valid, alpha, torch.zeros_like(alpha))
            Tafter = torch.cumprod(1.0 - ae, 0)
            stop = valid & (Tafter < TMIN)
            first = torch.where(stop.any(0), stop.to(F).argmax(0), torch.full((len(xs),), len(ids)))
            incl = valid & (torch.arange(len(ids))[:, None] < first[None, :])
        ai = torch.where(incl, alpha, torch.zeros_like(alpha))
        Tb = torch.cat([torch.ones(1, len(xs), dtype=F), torch.cumprod(1.0 - ai, 0)[:-1]], 0)
        w = ai * Tb
        hit = mu[ids][:, None, :] + u[..., None] * (su[ids][:, None, None] * t_u[ids][:, None, :]) + \
            v[..., None] * (sv[ids][:, None, None] * t_v[ids][:, None, :])
        hh, ww, off = dims[ids, 0][:, None], dims[ids, 1][:, None], dims[ids, 2][:, None]
        has = (hh * ww > 0)
        xr = hh.to(F) * (uv0[ids][:, None, 0] + ((hit - mu[ids][:, None, :]) * um[ids][:, None, :]).sum(-1))
        yr = ww.to(F) * (uv0[ids][:, None, 1] + ((hit - mu[ids][:, None, :]) * vm[ids][:, None, :]).sum(-1))
        xc = torch.minimum(torch.clamp(xr, min=0.0), (hh - 1).clamp(min=0).to(F))
        yc = torch.minimum(torch.clamp(yr, min=0.0), (ww - 1).clamp(min=0).to(F))
        i0, j0 = xc.detach().floor().long(), yc.detach().floor().long()
        i1, j1 = torch.minimum(i0 + 1, (hh - 1).clamp(min=0)), torch.minimum(j0 + 1, (ww - 1).clamp(min=0))
        ax, ay = (xc - i0.to(F))[..., None], (yc - j0.to(F))[..., None]
        if tex.shape[0]:
            fetch = lambda i, j: tex[torch.where(has, off + i * ww + j, torch.zeros_like(i)).clamp(0, tex.shape[0] - 1)]  # noqa: E731
            val = (1 - ax) * ((1 - ay) * fetch(i0, j0) + ay * fetch(i0, j1)) + ax * ((1 - ay) * fetch(i1, j0) + ay * fetch(i1, j1))
            val = torch.where(has[..., None], val, torch.zeros_like(val))
        else:
            val = torch.zeros(len(ids), len(xs), C, dtype=F)
        rows["img"].append((w[..., None] * rgb[ids][:, None, :]).sum(0))
        rows["alpha"].append(1.0 - torch.prod(1.0 - ai, 0))
        rows["depth"].append((w * torch.where(incl, z, torch.ones_like(z))).sum(0))
        rows["tex"].append((w[..., None] * val).sum(0))
        rows["normal"].append((w[..., None] * nrm[ids][:, None, :]).sum(0))
        pix_all.append(ys * W + xs)
    pix = torch.cat(pix_all)
    for k in out:
        flat = out[k].reshape(H * W, *out[k].shape[2:]).index_put((pix,), torch.cat(rows[k], 0))
        out[k] = flat.reshape(out[k].shape)
    return out


@pytest.mark.parametrize("n_texels,keys", [
    # 2DGS mode: every gradient
    (0, ("rgbs", "opacities", "means", "scales", "quats", "centers")),
    # textured: the oracle takes the texel cell of each pair from the fp32 pass (what the kernels see), this
    # restatement from float64, so where a sample point lies within an fp32 ulp of a texel edge the two bilinear
    # slopes differ -- the coordinate gradients (means, scales, quats) are compared on the 2DGS scene only
    (3000, ("rgbs", "opacities", "texture", "centers")),
])
def test_world_space_ray_restatement_gradients_match_oracle(n_texels, keys):
    """The oracle's fp64 autograd (of the kernels' formulation) against autograd of the world-space restatement, for
    the same upstream gradients, both in float64: equal to 1e-10 of each gradient's largest element."""
    from helpers import DIFF, upstream

    case = make_case(n=60, n_texels=n_texels, H=32, W=32, seed=21)
    inp = case.inp
    mine = {k: getattr(inp, k).detach().clone().double().requires_grad_(True) for k in DIFF}
    theirs = {k: getattr(inp, k).detach().clone().double().requires_grad_(True) for k in DIFF}
    for k, t in theirs.items():
        setattr(inp, k, t)
    _, o64, aux = O.rasterize(inp)
    up = upstream(32, 32, case.C, 5, aux["margin"] < FLIP_MARGIN)
    names = ("img", "alpha", "depth", "tex", "normal")
    sum((o64[k] * up[k].double()).sum() for k in names).backward()
    ref = ray_render_torch(inp, mine)
    sum((ref[k] * up[k].double()).sum() for k in names).backward()
    for k in names:
        assert float((ref[k] - o64[k]).detach().abs().max()) < 1e-10, k
    for k in keys:
        g, r = theirs[k].grad, mine[k].grad
        scale = float(r.abs().max())
        assert scale > 0, k
        assert float((g - r).abs().max()) <= 1e-10 * scale, f"{k}: {float((g - r).abs().max()):.3e} vs {scale:.3e}"
