"""Raster output conventions pinned by the REFERENCE's own code (tests/golden/make_conventions_golden.py).

The GStex_cuda kernels are absent from the reference, so the raster itself is parity-unpinned; these tests pin the
conventions its consumers fix:
  * pixel centre (x + 0.5, y + 0.5) and view-space z depth: the reference's depths_to_points (gstex.py:122-149,
    +0.5 at :138-139, "don't use view depth" at :145-146) puts the rendered depth / alpha of a plane back ON the
    plane (residual ~1e-6), where integer pixel coordinates would miss it by ~1e-2;
  * world-space normals facing the camera: the reference's depth_to_normal (gstex.py:151-161), as its normal loss
    uses it (gstex.py:1218-1220, 1316), agrees with the rendered normal in direction and sign;
  * the same with the AA low-pass (settings bit 9) on;
  * texel placement and the bilinear lookup: texel values a linear ramp in the reference's own texel uv
    (texture_dims_to_query, jagged_texture.py:23-34) render as that ramp at each pixel's uv (get_uv_mapping,
    gstex.py:975-990, of the hit point depths_to_points gives);
  * the composite (gstex.py:1204-1205) and the loss terms of get_loss_dict (gstex.py:1301-1322).
CPU tests: the oracle against the golden; -m gpu tests: the HIP path against the same golden.
"""
import os

import numpy as np
import pytest
import torch

from oracle import raster as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "conventions.npz")


@pytest.fixture(scope="module")
def z():
    with np.load(GOLD, allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def _plane_inputs(z, aa=False):
    H, W = (int(v) for v in z["plane_hw"])
    fx, fy, cx, cy = (float(v) for v in z["plane_intr"])
    vm = torch.from_numpy(z["plane_viewmat"])
    c2w = torch.from_numpy(z["plane_c2w"])
    cam = O.Camera(vm, fx, fy, cx, cy, H, W, 16, c2w[:3, 3])
    means = torch.from_numpy(z["plane_means"])
    scales = torch.from_numpy(z["plane_scales"])
    quats = torch.from_numpy(z["plane_quats"])
    opac = torch.from_numpy(z["plane_opacities"])
    n = means.shape[0]
    centers, extents = O.aabb_2d(means, scales, 1.0, quats, cam)
    _, depths = O.project_points(means, cam)
    inp = O.RasterInputs(torch.zeros((n, 3), dtype=torch.int32), centers, extents, depths, torch.full((n, 3), 0.5),
                         opac, means, scales, 1.0, quats, torch.full((n, 1, 2), 0.5), torch.zeros((n, 1, 3)),
                         torch.zeros((n, 1, 3)), torch.zeros((0, 3)), cam,
                         settings=int(z["plane_aa_settings" if aa else "plane_settings"][0]))
    return inp, (vm, c2w, fx, fy, cx, cy, H, W)


def _tex_inputs(z):
    H, W = (int(v) for v in z["tex_hw"])
    fx, fy, cx, cy = (float(v) for v in z["tex_intr"])
    vm = torch.from_numpy(z["tex_viewmat"])
    c2w = torch.from_numpy(z["tex_c2w"])
    cam = O.Camera(vm, fx, fy, cx, cy, H, W, 16, c2w[:3, 3])
    t = {k: torch.from_numpy(z["tex_" + k]) for k in ("means", "scales", "quats", "opacities", "dims", "texture",
                                                        "uv0", "umap", "vmap")}
    n = t["means"].shape[0]
    centers, extents = O.aabb_2d(t["means"], t["scales"], 1.0, t["quats"], cam)
    _, depths = O.project_points(t["means"], cam)
    inp = O.RasterInputs(t["dims"], centers, extents, depths, torch.full((n, 3), 0.5), t["opacities"], t["means"],
                         t["scales"], 1.0, t["quats"], t["uv0"], t["umap"], t["vmap"], t["texture"], cam,
                         settings=int(z["tex_settings"][0]))
    return inp, (vm, c2w, fx, fy, cx, cy, H, W)


def _hip_render(inp, vm, c2w, fx, fy, cx, cy, H, W):
    import gstex_cuda

    dev = "cuda"
    d = lambda t: t.detach().to(dev).contiguous()  # noqa: E731
    n = inp.means.shape[0]
    C = inp.texture.shape[1]
    nth = O.num_tiles_hit(inp.centers, inp.extents, H, W)
    outs = gstex_cuda.texture_gaussians(
        (n, 1, C), d(inp.texture_dims), d(inp.centers), d(inp.extents), d(inp.depths), d(nth), d(inp.rgbs),
        d(inp.opacities), d(inp.means), d(inp.scales), 1.0, d(inp.quats), d(inp.uv0), d(inp.umap), d(inp.vmap),
        d(inp.texture), d(vm), d(c2w), fx, fy, cx, cy, H, W, 16, inp.settings)
    return {"depth": outs[1].cpu(), "alpha": outs[3].cpu(), "tex": outs[4].cpu(), "normal": outs[5].cpu()}


def _interior(alpha):
    from scipy.ndimage import binary_erosion

    m = binary_erosion(alpha > 0.999)
    m[0, :] = m[-1, :] = m[:, 0] = m[:, -1] = False
    return m


def test_reference_points_lie_on_the_plane(z):
    """depths_to_points (reference) of depth / alpha: on the plane to ~1e-6, vs >= 1e-2 for integer centres."""
    inside = z["plane_alpha"] > 0.999
    assert inside.mean() > 0.5
    n = z["plane_normal"].astype(np.float64)
    res = np.abs(z["plane_ref_points"].astype(np.float64) @ n)[inside]
    ctrl = np.abs(z["plane_ref_points_intcentre"].astype(np.float64) @ n)[inside]
    assert res.max() < 1e-5, res.max()
    assert ctrl.min() > 1e-3 and ctrl.min() > 1000 * res.max(), (ctrl.min(), res.max())


def test_reference_estimated_normals_match_rendered(z):
    """depth_to_normal (reference, on the raw depth as gstex.py:1220 calls it) == the rendered normal's direction,
    same sign (both face the camera, world space).  The raw depth carries the (1 - T) factor (T in [1e-4, 1e-3]),
    so the agreement is ~1e-4 in cos, not exact."""
    m = _interior(z["plane_alpha"])
    assert m.sum() > 1000
    est = z["plane_ref_est_normal"].astype(np.float64)
    rn = z["plane_rnormal"].astype(np.float64)
    rnn = rn / np.linalg.norm(rn, axis=-1, keepdims=True).clip(1e-30)
    cos = (est * rnn).sum(-1)[m]
    assert cos.min() > 0.999 and np.median(cos) > 0.99995, (cos.min(), np.median(cos))
    # the rendered normal is the plane's (world space) oriented toward the camera
    campos = z["plane_c2w"][:3, 3].astype(np.float64)
    n = z["plane_normal"].astype(np.float64)
    assert np.all(np.abs(rnn[m] @ n) > 1 - 1e-6)
    assert np.all(rnn[m] @ campos > 0)  # the plane passes through the origin: facing the camera


def test_oracle_renders_the_golden_plane(z):
    inp, _ = _plane_inputs(z)
    o32, _, _ = O.rasterize(inp)
    for k, g in (("depth", "plane_depth"), ("alpha", "plane_alpha"), ("normal", "plane_rnormal")):
        np.testing.assert_array_equal(o32[k].numpy(), z[g], err_msg=k)


def test_reference_points_lie_on_the_aa_plane(z):
    """The same plane with the AA low-pass on (settings bit 9, the reference's default): the reference's
    depths_to_points puts >= 99 % of the interior pixels on the plane to 1e-5 and its depth_to_normal agrees with the
    rendered normals.  (The few off the plane -- 14 of 3,212 -- lie next to a splat's AABB centre, where 2 |centre -
    pixel|^2 undercuts the ray-splat distance and the 2DGS screen-space branch, depth = the centre's, takes over.)"""
    inside = z["plane_aa_alpha"] > 0.999
    assert inside.mean() > 0.5
    n = z["plane_normal"].astype(np.float64)
    res = np.abs(z["plane_aa_ref_points"].astype(np.float64) @ n)[inside]
    assert (res < 1e-5).mean() > 0.99, (res < 1e-5).mean()
    assert np.abs(z["plane_aa_depth"] - z["plane_depth"]).max() > 0  # the bit changed some pixels
    m = _interior(z["plane_aa_alpha"])
    est = z["plane_aa_ref_est_normal"].astype(np.float64)
    rn = z["plane_aa_rnormal"].astype(np.float64)
    cos = (est * (rn / np.linalg.norm(rn, axis=-1, keepdims=True).clip(1e-30))).sum(-1)[m]
    assert cos.min() > 0.999 and np.median(cos) > 0.99995, (cos.min(), np.median(cos))


def test_textured_render_is_the_reference_texel_ramp(z):
    """Texel values a linear ramp in the reference's texel uv (texture_dims_to_query, jagged_texture.py:23-34): the
    rendered texture / alpha of each pixel equals the ramp at that pixel's uv (reference get_uv_mapping of the hit
    point the reference's depths_to_points gives) to ~1e-6 -- texels corner-aligned at (i / h, j / w), bilinear --
    while texel-centred placement ((i + 0.5) / h) misses by >= 5e-3."""
    m = z["tex_mask"]
    assert m.sum() > 500
    val = z["tex_render"] / np.maximum(z["tex_alpha"], 1e-30)[..., None]
    err = np.abs(val - z["tex_ref_pred"])[m]
    ctrl = np.abs(val - z["tex_ref_pred_centre"])[m]
    assert err.max() < 1e-5, err.max()
    assert ctrl.min() > 1e-3 and ctrl.min() > 100 * err.max(), (ctrl.min(), err.max())


def test_oracle_renders_the_golden_aa_plane_and_textured_splats(z):
    inp, _ = _plane_inputs(z, aa=True)
    o32, _, _ = O.rasterize(inp)
    for k, g in (("depth", "plane_aa_depth"), ("alpha", "plane_aa_alpha"), ("normal", "plane_aa_rnormal")):
        np.testing.assert_array_equal(o32[k].numpy(), z[g], err_msg=k)
    inp, _ = _tex_inputs(z)
    o32, _, _ = O.rasterize(inp)
    for k, g in (("tex", "tex_render"), ("alpha", "tex_alpha"), ("depth", "tex_depth")):
        np.testing.assert_array_equal(o32[k].numpy(), z[g], err_msg=k)


def test_composite_and_loss_terms_match_reference(z):
    """The composite (gstex.py:1204-1205) as GStexTrainer.render forms it, and the loss combination of
    get_loss_dict with the golden's stubbed SSIM value."""
    img, tex, alpha = (torch.from_numpy(z[k]) for k in ("loss_img", "loss_tex", "loss_alpha"))
    bg, gt = torch.from_numpy(z["loss_bg"]), torch.from_numpy(z["loss_gt"])
    rgb = torch.clamp(img + tex[:, :, 0:3] + (1 - alpha[:, :, None]) * bg[None, None, :], 0.0, 1.0)  # model.py
    np.testing.assert_array_equal(rgb.numpy(), z["loss_rgb"])
    l1 = torch.abs(gt - rgb).mean()
    assert abs(float(l1) - float(z["loss_l1"][0])) < 1e-7
    lam_ssim, lam_reg, lam_normal = (float(v) for v in z["loss_lambdas"])
    main = (1 - lam_ssim) * l1 + lam_ssim * (1 - float(z["loss_ssim_stub"][0]))
    assert abs(float(main) - float(z["loss_main"][0])) < 1e-7
    normal, est, reg = (torch.from_numpy(z[k]) for k in ("loss_normal", "loss_est", "loss_reg"))
    nl = lam_normal * torch.mean(alpha - torch.sum(normal * est, dim=-1))
    assert abs(float(nl) - float(z["loss_normal_loss"][0])) < 1e-7
    assert abs(float(lam_reg * reg.mean()) - float(z["loss_reg_loss"][0])) < 1e-7


# ------------------------------------------------------------------------------------------ HIP path
@pytest.mark.gpu
def test_hip_plane_depth_normal_match_golden(z):
    """The HIP rasterizer's depth / alpha / normal of the plane: within the forward tolerance of the golden, so the
    reference's depths_to_points / depth_to_normal see the same geometry from the HIP path."""
    from helpers import TOL_ABS, TOL_REL

    for aa in (False, True):
        inp, geom = _plane_inputs(z, aa=aa)
        got = _hip_render(inp, *geom)
        p = "plane_aa_" if aa else "plane_"
        for k in ("depth", "alpha", "normal"):
            ref = torch.from_numpy(z[p + ("rnormal" if k == "normal" else k)]).double()
            err = (got[k].double() - ref).abs()
            assert bool((err <= TOL_ABS + TOL_REL * ref.abs()).all()), f"{p}{k}: max err {float(err.max()):.3e}"


@pytest.mark.gpu
def test_hip_textured_splats_match_golden_and_reference_ramp(z):
    """The HIP path on the textured golden: within the forward tolerance of the golden render, and its texture /
    alpha equal to the reference-predicted texel ramp (test_textured_render_is_the_reference_texel_ramp)."""
    from helpers import TOL_ABS, TOL_REL

    inp, geom = _tex_inputs(z)
    got = _hip_render(inp, *geom)
    for k, g in (("tex", "tex_render"), ("alpha", "tex_alpha"), ("depth", "tex_depth")):
        ref = torch.from_numpy(z[g]).double()
        err = (got[k].double() - ref).abs()
        assert bool((err <= TOL_ABS + TOL_REL * ref.abs()).all()), f"{k}: max err {float(err.max()):.3e}"
    m = z["tex_mask"]
    val = got["tex"].numpy() / np.maximum(got["alpha"].numpy(), 1e-30)[..., None]
    assert np.abs(val - z["tex_ref_pred"])[m].max() < 1e-5


@pytest.mark.gpu
def test_hip_composite_and_l1_match_reference(z):
    """The fused loss kernel (gstex_amd.loss, ssim_lambda = 0: the loss is L1) against the reference's composite and
    L1 (gstex.py:1204-1205, 1301)."""
    from gstex_amd.loss import photometric_loss

    dev = "cuda"
    img, tex, alpha, bg, gt = (torch.from_numpy(z[k]).to(dev).contiguous()
                               for k in ("loss_img", "loss_tex", "loss_alpha", "loss_bg", "loss_gt"))
    loss, rgb = photometric_loss(img, tex, alpha, bg, gt, ssim_lambda=0.0)
    np.testing.assert_allclose(rgb.cpu().numpy(), z["loss_rgb"], rtol=0, atol=1e-7)
    assert abs(float(loss) - float(z["loss_l1"][0])) < 1e-6 * max(1.0, float(z["loss_l1"][0]))


def test_depth_to_normal_and_geometry_loss_restate_reference(z):
    """gstex_amd.loss.depths_to_points / depth_to_normal / geometry_loss (GStexTrainer's lambda_normal / lambda_reg
    terms) against the reference's own functions' outputs in the golden (gstex.py:122-161, 1313-1317)."""
    from gstex_amd.loss import depth_to_normal, depths_to_points, geometry_loss, scheduled

    vm, c2w = torch.from_numpy(z["plane_viewmat"]), torch.from_numpy(z["plane_c2w"])
    fx, fy, cx, cy = (float(v) for v in z["plane_intr"])
    depth, alpha = torch.from_numpy(z["plane_depth"]), torch.from_numpy(z["plane_alpha"])
    inside = alpha > 0.999
    pts = depths_to_points((depth / alpha.clamp(min=1e-30))[..., None], vm, c2w, fx, fy, cx, cy)
    np.testing.assert_allclose(pts.numpy()[inside.numpy()], z["plane_ref_points"][inside.numpy()], rtol=0, atol=2e-6)
    est = depth_to_normal(depth[..., None], vm, c2w, fx, fy, cx, cy)
    ref = torch.from_numpy(z["plane_ref_est_normal"])
    m = torch.from_numpy(_interior(z["plane_alpha"]))
    assert float((est - ref)[m].abs().max()) < 1e-4
    assert float(est[0].abs().max()) == 0.0 and float(est[:, -1].abs().max()) == 0.0  # zero border
    lam_ssim, lam_reg, lam_normal = (float(v) for v in z["loss_lambdas"])
    normal, est_l, reg = (torch.from_numpy(z[k]) for k in ("loss_normal", "loss_est", "loss_reg"))
    a = torch.from_numpy(z["loss_alpha"])
    g = geometry_loss(a, normal, est_l, reg, lam_normal, lam_reg)
    assert abs(float(g) - float(z["loss_normal_loss"][0] + z["loss_reg_loss"][0])) < 1e-7
    assert scheduled([0.0, 0.05, 7000], 6999) == 0.0 and scheduled([0.0, 0.05, 7000], 7000) == 0.05
    assert scheduled(3, 0) == 3.0
