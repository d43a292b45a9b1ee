"""GStexTrainer.eval_render (one binning, 3-channel raster calls) against the reference's formulation of the eval
render: three 6-channel texture_gaussians calls on [SH2RGB(texture_dc), 0, 0, 0] / [edit or 0, 0, 0, 0]
(gstex.py:1086-1203), written out here with the public API."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _reference_eval(tr, view, edit_texture=None):
    import gstex_cuda
    from gstex_amd import ops
    from gstex_amd.activations import activate, sh_rest
    from gstex_amd.charts import SH2RGB

    means = tr.means.detach()
    quats, scales, opacities, uv0, umap, vmap, viewdirs = activate(
        means, tr.quats.detach(), tr.scales.detach(), tr.opacities.detach(), tr.mappings, view.c2w[:3, 3])
    if tr.fix_init and tr.sh_degree > 0:
        viewdirs = torch.stack([viewdirs[:, 0], -viewdirs[:, 2], viewdirs[:, 1]], -1)
    intr = (view.fx, view.fy, view.cx, view.cy)
    _, depths = ops.project_points(means, view.viewmat, intr)
    centers, extents = ops.get_aabb_2d(means, scales, 1, quats, view.viewmat, intr)
    nth = ops.get_num_tiles_hit_2d(centers, extents, view.H, view.W, 16)
    n = means.shape[0]
    rgbs = sh_rest(tr.sh_degree_now(), viewdirs, tr.features_rest.detach())
    tex6 = torch.zeros((tr.texture_dc.shape[0], 6), device=DEV)
    tex6[:, 0:3] = SH2RGB(tr.texture_dc.detach())
    bgz = torch.zeros_like(tr.background)

    def tg(cr, ct, co, st):
        return gstex_cuda.texture_gaussians(
            (n, 1, 6), tr.texture_dims, centers, extents, depths, nth, cr, co, means, scales, 1, quats, uv0, umap,
            vmap, ct, view.viewmat, view.c2w, view.fx, view.fy, view.cx, view.cy, view.H, view.W, 16, st,
            background=bgz)

    img, depth, reg, alpha, tex, normal = tg(rgbs, tex6, opacities, tr.settings)
    upd = torch.zeros_like(tex6)
    upd[:, 3:] = tex6[:, 3:]
    if edit_texture is not None:
        upd[:, :3] = edit_texture
    test_op = opacities.clone()
    test_op[test_op <= 0.5] = 0.0
    test_op[test_op > 0.2] = 1.0
    t_out = tg(tr.test_colors, upd, test_op, tr.settings)
    n_out = tg(tr.test_colors, upd, opacities, tr.settings | (1 << 15))
    bg = tr.background[None, None, :]
    rgb = torch.clamp(img + tex[..., 0:3] + (1 - alpha[..., None]) * bg, 0.0, 1.0)
    return dict(rgb=rgb, depth=depth, alpha=alpha, normal=normal,
                test_img=t_out[0] + (1 - t_out[3][..., None]) * bg,
                uv_im=torch.clamp(t_out[4][..., 3:6] + (1 - t_out[3][..., None]) * bg, 0.0, 1.0),
                edit_img=torch.clamp(img + n_out[4][..., :3] + (1 - alpha[..., None]) * bg, 0.0, 1.0),
                clean_normal_img=torch.clamp(0.5 * (n_out[5] + 1) + (1 - alpha[..., None]) * bg, 0.0, 1.0))


@pytest.mark.parametrize("edit", [False, True])
def test_eval_render_matches_six_channel_calls(edit):
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    sc = make_scene(4000, 80000, seed=5)
    tr = GStexTrainer(sc, DEV, start_step=3000)
    view = sphere_view(2, 120, 152).to(DEV)
    edit_tex = None
    if edit:
        g = torch.Generator().manual_seed(7)
        edit_tex = torch.rand((tr.texture_dc.shape[0], 3), generator=g).to(DEV)
    with torch.no_grad():
        got = tr.eval_render(view, edit_texture=edit_tex)
        ref = _reference_eval(tr, view, edit_texture=edit_tex)
    assert float(ref["alpha"].max()) > 0.5
    for k in ref:
        # texture values: SH2RGB applied after the bilinear mix instead of before (last-bit rounding)
        err = float((got[k] - ref[k]).abs().max())
        assert err <= 2e-5 * max(1.0, float(ref[k].abs().max())), f"{k}: {err:.3e}"
