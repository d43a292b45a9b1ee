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
