"""Pin the rasterizer's output conventions with the REFERENCE's own code.

Run in the build container only (reads /root/reference, which the GPU box does not have):
    python tests/golden/make_conventions_golden.py
Writes tests/golden/conventions.npz.  The GStex_cuda kernels are absent, so the raster itself cannot be pinned;
what CAN run is the reference Python that consumes the raster outputs.  Functions are AST-extracted from the source
text (like make_golden.py) and exec'd; only inputs and outputs are committed.

1. Plane scene (depth / normal conventions), without and (1b) with the AA bit 9: a tilted plane tiled with opaque, overlapping coplanar splats (2DGS
   mode, no texels) is rendered by the CPU oracle (oracle/raster.py, the restatement the HIP kernels are tested
   against).  The rendered depth goes through the reference's
       depths_to_points / depth_to_normal      nerfstudio/models/gstex.py:122-161
   exactly as its normal loss does (gstex.py:1218-1220, 1316).  Committed: the scene, the oracle's depth / alpha /
   normal, the reference's estimated normals and the reference's 3-D points of depth / alpha.  The tests check that
   the reference's points lie on the plane (pins pixel centre +0.5 and view-z depth, gstex.py:138-139, 145-146) and
   that its estimated normals equal the rendered ones in direction AND sign (pins world-space normals oriented to
   the camera, gstex.py:1316).  As a control, the points the same code gives with the principal point moved by half
   a pixel (i.e. a rasterizer sampling integer pixel coordinates, as 2DGS does) are stored too.
1c. Textured splats (texel placement and bilinear lookup): see textured_scene().
2. Composite + loss: the background composite (gstex.py:1204-1205, two statements of get_outputs) and
   GStexModel.get_loss_dict (gstex.py:1277-1322, with composite_with_background gstex.py:1249-1260) on seeded
   random raster outputs.  pytorch_msssim is absent, so self.ssim is a stub returning a fixed value; the golden pins
   the composite, L1, the 0.8 / 0.2 combination and the normal / distortion terms.
"""
import ast
import math
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = "/root/reference/nerfstudio/models/gstex.py"
REF_JT = "/root/reference/nerfstudio/models/jagged_texture.py"
OUT = os.path.join(HERE, "conventions.npz")

SSIM_STUB = 0.8125  # self.ssim(...) in the loss golden (pytorch_msssim is not importable here)


def extract_functions(path, names):
    src = open(path).read()
    tree = ast.parse(src)
    found = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name in names and node.name not in found:
            found[node.name] = ast.get_source_segment(src, node)
    assert set(found) == set(names), set(names) - set(found)
    return found


def extract_composite(path):
    """The two statements of GStexModel.get_outputs that form the training image (gstex.py:1204-1205)."""
    src = open(path).read()
    tree = ast.parse(src)
    fn = next(n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name == "get_outputs")
    stmts = [n for n in fn.body if isinstance(n, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "rgb"
                                                                      for t in n.targets)]
    assert len(stmts) == 2, len(stmts)
    return "\n".join(ast.get_source_segment(src, n) for n in stmts), [n.lineno for n in stmts]


def plane_scene(H=64, W=64, view=1, tilt_deg=35.0, spacing=0.1, sigma=0.1, opacity=0.95, settings=None):
    from scipy.spatial.transform import Rotation

    from gstex_amd.scene import sphere_view
    from oracle import raster as O

    v = sphere_view(view, H, W)
    c2w = v.c2w.double()
    campos = c2w[:3, 3]
    fwd = -campos / campos.norm()  # the camera looks at the origin
    # plane normal: the direction to the camera tilted by tilt_deg about the camera's x axis
    ax = c2w[:3, 0]
    n_p = torch.from_numpy(Rotation.from_rotvec((math.radians(tilt_deg) * ax).numpy()).apply((-fwd).numpy()))
    t1 = torch.linalg.cross(n_p, ax)
    t1 = t1 / t1.norm()
    t2 = torch.linalg.cross(n_p, t1)
    R = torch.stack([t1, t2, n_p], 1)  # columns t_u, t_v, t_w
    q_xyzw = Rotation.from_matrix(R.numpy()).as_quat()
    q = torch.tensor([q_xyzw[3], q_xyzw[0], q_xyzw[1], q_xyzw[2]], dtype=torch.float64)
    g = torch.arange(-14, 15, dtype=torch.float64) * spacing
    a, b = torch.meshgrid(g, g, indexing="ij")
    means = (a.reshape(-1, 1) * t1 + b.reshape(-1, 1) * t2).float()
    n = means.shape[0]
    quats = q.float()[None].repeat(n, 1)
    scales = torch.tensor([sigma, sigma, 1e-5 * sigma], dtype=torch.float32)[None].repeat(n, 1)
    opac = torch.full((n, 1), opacity)
    cam = O.Camera(v.viewmat, v.fx, v.fy, v.cx, v.cy, H, W, 16, v.c2w[:3, 3])
    centers, extents = O.aabb_2d(means, scales, 1.0, quats, cam)
    _, depths = O.project_points(means, cam)
    dims = torch.zeros((n, 3), dtype=torch.int32)
    uv0 = torch.full((n, 1, 2), 0.5)
    umap = torch.zeros((n, 1, 3))
    vmap = torch.zeros((n, 1, 3))
    rgbs = torch.full((n, 3), 0.5)
    # without the AA low-pass (bit 9): every hit lies on the splat plane (with it, a pixel next to the AABB centre can
    # take the 2DGS screen-space branch, whose depth is the splat centre's), so the geometry is exact
    inp = O.RasterInputs(dims, centers, extents, depths, rgbs, opac, means, scales, 1.0, quats, uv0, umap, vmap,
                         torch.zeros((0, 3)), cam, settings=O.SETTING_DIST_REG if settings is None else settings)
    o32, _, _ = O.rasterize(inp)
    return v, inp, o32, n_p.float()


def textured_scene(ns, H=96, W=96, view=1, sigma_px=3.5, opacity=0.9, settings=None):
    """Three fronto-parallel splats, well apart (no pixel sees two), each with its own texel block whose values are a
    linear ramp in the REFERENCE's texel uv (texture_dims_to_query, jagged_texture.py:23-34): value_c(i, j) =
    a_c u_ij + b_c v_ij + c_c.  Bilinear interpolation reproduces a linear function exactly, so a pixel's texture
    value is the ramp at the pixel's own uv -- uv0 + ((X - mu) . umap, (X - mu) . vmap) with (uv0, umap, vmap) from
    the reference's get_uv_mapping (gstex.py:975-990) and X the hit point the reference's depths_to_points gives
    (gstex.py:122-149) -- wherever that uv lies inside the block (clamped edges aside).  This pins where texel (i, j)
    sits (corner-aligned at (i/h, j/w)) and the bilinear lookup, with the default settings (bits 9, 10)."""
    from scipy.spatial.transform import Rotation

    from gstex_amd.scene import sphere_view
    from oracle import raster as O

    if settings is None:
        settings = O.SETTING_AA_BLUR | O.SETTING_DIST_REG
    v = sphere_view(view, H, W)
    c2w = v.c2w.double()
    campos = c2w[:3, 3]
    dist = float(campos.norm())  # the camera looks at the origin
    right, down, fwd = c2w[:3, 0], c2w[:3, 1], c2w[:3, 2]
    offs = [(-24.0, -10.0), (22.0, -12.0), (0.0, 22.0)]  # pixel offsets of the centres from the principal point
    means = torch.stack([campos + dist * (fwd + (ox / v.fx) * right + (oy / v.fy) * down) for ox, oy in offs]).float()
    n = means.shape[0]
    q_xyzw = Rotation.from_matrix(c2w[:3, :3].numpy()).as_quat()  # splat frame = camera axes: fronto-parallel
    quats = torch.tensor([q_xyzw[3], q_xyzw[0], q_xyzw[1], q_xyzw[2]], dtype=torch.float32)[None].repeat(n, 1)
    sig = sigma_px * dist / v.fx
    scales = torch.tensor([sig, sig, 1e-5 * sig], dtype=torch.float32)[None].repeat(n, 1)
    opac = torch.full((n, 1), opacity)
    hw = torch.tensor([[8, 6], [5, 9], [7, 7]], dtype=torch.int32)
    cnt = hw[:, 0] * hw[:, 1]
    dims = torch.cat([hw, (torch.cumsum(cnt, 0) - cnt).to(torch.int32)[:, None]], 1).to(torch.int32)
    ids, uvq = ns["texture_dims_to_query"](dims)  # the reference's texel uv (i / h, j / w)
    g = torch.Generator().manual_seed(404)
    coef = torch.rand((n, 3, 3), generator=g) - 0.5  # [splat, channel, (a, b, c)]
    coef[:, :, 2] += 0.5
    tex = (coef[ids, :, 0] * uvq[:, 0:1] + coef[ids, :, 1] * uvq[:, 1:2] + coef[ids, :, 2]).float().contiguous()
    mappings = torch.full((n, 2), 1.0 / (6.0 * sig))  # u, v in [0, 1] over +-3 sigma
    uv0, umap, vmap = ns["get_uv_mapping"](None, means, quats, mappings)
    cam = O.Camera(v.viewmat, v.fx, v.fy, v.cx, v.cy, H, W, 16, v.c2w[:3, 3])
    centers, extents = O.aabb_2d(means, scales, 1.0, quats, cam)
    _, depths = O.project_points(means, cam)
    inp = O.RasterInputs(dims, centers, extents, depths, torch.full((n, 3), 0.5), opac, means, scales, 1.0, quats,
                         uv0.float(), umap.float(), vmap.float(), tex, cam, settings=settings)
    o32, _, _ = O.rasterize(inp)
    return v, inp, o32, coef


def main():
    sys.path.insert(0, "/root/reference")
    from oracle import raster as O  # noqa: F401  (test infrastructure)

    fns = extract_functions(REF, ["depths_to_points", "depth_to_normal", "get_loss_dict",
                                  "composite_with_background", "get_uv_mapping"])
    fns.update(extract_functions(REF_JT, ["texture_dims_to_query"]))
    from typing import Dict, Optional  # annotations of the extracted signatures

    from nerfstudio.utils.rotations import quaternion_to_matrix  # pure torch (as make_golden.py)

    ns = {"torch": torch, "np": np, "math": math, "Dict": Dict, "Optional": Optional,
          "quat_to_rotmat": quaternion_to_matrix}
    for code in fns.values():
        exec(code, ns)
    out = {}

    # ---- 1. plane scene
    H = W = 64
    v, inp, o32, n_p = plane_scene(H, W)
    depth = o32["depth"][..., None]
    alpha = o32["alpha"][..., None]
    intr = (v.fx, v.fy, v.cx, v.cy)
    est = ns["depth_to_normal"](depth, v.viewmat, v.c2w, intr, H, W)
    zn = torch.where(alpha > 0, depth / alpha.clamp(min=1e-12), torch.zeros_like(depth))
    pts = ns["depths_to_points"](zn, v.viewmat, v.c2w, intr, H, W)
    # control: the same depth placed on the rays through the integer pixel coordinates
    pts_int = ns["depths_to_points"](zn, v.viewmat, v.c2w, (v.fx, v.fy, v.cx + 0.5, v.cy + 0.5), H, W)
    out.update(
        plane_means=inp.means.numpy(), plane_scales=inp.scales.numpy(), plane_quats=inp.quats.numpy(),
        plane_opacities=inp.opacities.numpy(), plane_viewmat=v.viewmat.numpy(), plane_c2w=v.c2w.numpy(),
        plane_intr=np.array([v.fx, v.fy, v.cx, v.cy], dtype=np.float64), plane_hw=np.array([H, W]),
        plane_normal=n_p.numpy(), plane_settings=np.array([inp.settings]),
        plane_depth=o32["depth"].numpy(), plane_alpha=o32["alpha"].numpy(), plane_rnormal=o32["normal"].numpy(),
        plane_ref_est_normal=est.numpy(), plane_ref_points=pts.numpy(), plane_ref_points_intcentre=pts_int.numpy())

    # ---- 1b. the same plane with the AA low-pass (settings bit 9, the reference's default, gstex.py:1157): at this
    # splat size (sigma ~2 px) every pixel's ray-splat distance is below the low-pass one, so the render must stay on
    # the plane -- pins that bit 9 leaves well-resolved geometry alone (the low-pass branch itself, taken only under
    # splats below ~0.7 px, is pinned by the oracle tests alone)
    from oracle import raster as O

    va, inpa, oa, _ = plane_scene(H, W, settings=O.SETTING_AA_BLUR | O.SETTING_DIST_REG)
    da, aa = oa["depth"][..., None], oa["alpha"][..., None]
    zna = torch.where(aa > 0, da / aa.clamp(min=1e-12), torch.zeros_like(da))
    out.update(plane_aa_settings=np.array([inpa.settings]), plane_aa_depth=oa["depth"].numpy(),
               plane_aa_alpha=oa["alpha"].numpy(), plane_aa_rnormal=oa["normal"].numpy(),
               plane_aa_ref_est_normal=ns["depth_to_normal"](da, va.viewmat, va.c2w, intr, H, W).numpy(),
               plane_aa_ref_points=ns["depths_to_points"](zna, va.viewmat, va.c2w, intr, H, W).numpy())

    # ---- 1c. textured splats: texel values a linear ramp in the reference's texel uv
    vt, inpt, ot, coef = textured_scene(ns)
    Ht, Wt = vt.H, vt.W
    intr_t = (vt.fx, vt.fy, vt.cx, vt.cy)
    dt, at = ot["depth"][..., None], ot["alpha"][..., None]
    znt = torch.where(at > 0, dt / at.clamp(min=1e-12), torch.zeros_like(dt))
    X = ns["depths_to_points"](znt, vt.viewmat, vt.c2w, intr_t, Ht, Wt).reshape(Ht, Wt, 3).double()
    # the splat each pixel sees: the nearest projected centre (the splats are > 30 px apart)
    yy, xx = torch.meshgrid(torch.arange(Ht, dtype=torch.float64) + 0.5, torch.arange(Wt, dtype=torch.float64) + 0.5,
                            indexing="ij")
    cxy = inpt.centers.double()
    d2 = (xx[..., None] - cxy[:, 0]) ** 2 + (yy[..., None] - cxy[:, 1]) ** 2
    k = d2.argmin(-1)
    mu = inpt.means.double()[k]
    uv = inpt.uv0[:, 0, :].double()[k] + torch.stack([((X - mu) * inpt.umap[:, 0, :].double()[k]).sum(-1),
                                                      ((X - mu) * inpt.vmap[:, 0, :].double()[k]).sum(-1)], -1)
    cf = coef.double()[k]  # (H, W, 3, 3)
    pred = cf[..., 0] * uv[..., 0:1] + cf[..., 1] * uv[..., 1:2] + cf[..., 2]
    # control: texel (i, j) at the texel-centre uv ((i + 0.5) / h, (j + 0.5) / w) instead
    hwk = inpt.texture_dims[:, :2].double()[k]
    pred_c = cf[..., 0] * (uv[..., 0:1] - 0.5 / hwk[..., 0:1]) + cf[..., 1] * (uv[..., 1:2] - 0.5 / hwk[..., 1:2]) + cf[..., 2]
    m = 0.01
    mask = ((at[..., 0] > 0.02) & (uv[..., 0] > m) & (uv[..., 0] < (hwk[..., 0] - 1) / hwk[..., 0] - m)
            & (uv[..., 1] > m) & (uv[..., 1] < (hwk[..., 1] - 1) / hwk[..., 1] - m))
    out.update(tex_means=inpt.means.numpy(), tex_scales=inpt.scales.numpy(), tex_quats=inpt.quats.numpy(),
               tex_opacities=inpt.opacities.numpy(), tex_dims=inpt.texture_dims.numpy(), tex_texture=inpt.texture.numpy(),
               tex_uv0=inpt.uv0.numpy(), tex_umap=inpt.umap.numpy(), tex_vmap=inpt.vmap.numpy(),
               tex_viewmat=vt.viewmat.numpy(), tex_c2w=vt.c2w.numpy(),
               tex_intr=np.array([vt.fx, vt.fy, vt.cx, vt.cy], dtype=np.float64), tex_hw=np.array([Ht, Wt]),
               tex_settings=np.array([inpt.settings]), tex_render=ot["tex"].numpy(), tex_alpha=ot["alpha"].numpy(),
               tex_depth=ot["depth"].numpy(), tex_ref_pred=pred.numpy(), tex_ref_pred_centre=pred_c.numpy(),
               tex_mask=mask.numpy())

    # ---- 2. composite + loss
    comp_src, comp_lines = extract_composite(REF)
    g = torch.Generator().manual_seed(77)
    Hl, Wl = 24, 20
    out_img = torch.rand((Hl, Wl, 3), generator=g) * 0.8
    out_texture = torch.rand((Hl, Wl, 3), generator=g) * 0.6 - 0.1
    out_alpha = torch.rand((Hl, Wl), generator=g)
    background = torch.rand(3, generator=g)
    cns = {"torch": torch, "out_img": out_img, "out_texture": out_texture, "out_alpha": out_alpha,
           "background": background}
    exec(comp_src, cns)
    rgb = cns["rgb"]
    gt = torch.rand((Hl, Wl, 3), generator=g)
    normal = torch.randn((Hl, Wl, 3), generator=g)
    est_n = torch.nn.functional.normalize(torch.randn((Hl, Wl, 3), generator=g), dim=-1)
    reg = torch.rand((Hl, Wl, 1), generator=g)
    fake = types.SimpleNamespace()
    fake.config = types.SimpleNamespace(ssim_lambda=0.2, lambda_reg=0.3, lambda_normal=0.05)
    fake.step = 0
    fake.get_gt_img = lambda image: image
    fake.composite_with_background = types.MethodType(ns["composite_with_background"], fake)
    fake.ssim = lambda a, b: torch.tensor(SSIM_STUB)
    outputs = {"rgb": rgb, "background": background, "accumulation": out_alpha[..., None], "normal_im": normal,
               "estimated_normals": est_n, "reg": reg}
    ld = ns["get_loss_dict"](fake, outputs, {"image": gt})
    out.update(loss_img=out_img.numpy(), loss_tex=out_texture.numpy(), loss_alpha=out_alpha.numpy(),
               loss_bg=background.numpy(), loss_gt=gt.numpy(), loss_normal=normal.numpy(), loss_est=est_n.numpy(),
               loss_reg=reg.numpy(), loss_rgb=rgb.numpy(), loss_l1=np.array([float(torch.abs(gt - rgb).mean())]),
               loss_main=np.array([float(ld["main_loss"])]), loss_normal_loss=np.array([float(ld["normal_loss"])]),
               loss_reg_loss=np.array([float(ld["reg_loss"])]), loss_ssim_stub=np.array([SSIM_STUB]),
               loss_lambdas=np.array([0.2, 0.3, 0.05]), composite_lines=np.array(comp_lines))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
