"""GStexTrainer's 2DGS regularisers (lambda_normal / lambda_reg / use_normal_loss, gstex.py:198-207, 1218-1222,
1313-1317) on the HIP path: the trainer's step equals the same loss assembled by hand from a geometry render
(photometric_loss + geometry_loss with the detached depth_to_normal estimate), gradient for gradient, and the
weights' [before, after, switch_step] schedule switches the geometry render on at its step."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_geometry_regularised_step_matches_manual_loss():
    from gstex_amd.loss import depth_to_normal, geometry_loss, photometric_loss
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    dev = torch.device("cuda", 0)
    sc = make_scene(3000, 60_000, seed=9)
    view = sphere_view(1, 96, 112).to(dev)
    gt = torch.rand((96, 112, 3), generator=torch.Generator().manual_seed(4)).to(dev)
    kw = dict(start_step=3000, lambda_normal=[0.0, 0.05, 3000], lambda_reg=0.02, use_normal_loss=True)
    auto = GStexTrainer(sc, dev, **kw)
    manual = GStexTrainer(sc, dev, start_step=3000)
    torch.use_deterministic_algorithms(True)  # splat gradients bitwise reproducible (row mode)
    try:
        auto.zero_grad()
        res = auto.forward_backward(view, gt)
        manual.zero_grad()
        out = manual.render(view, sh_degree_now=manual.sh_degree_now(), composite=False, geometry=True)
        loss, _ = photometric_loss(out["img"], out["tex"], out["alpha"], manual.background, gt.contiguous())
        est = depth_to_normal(out["depth"], view.viewmat, view.c2w, view.fx, view.fy, view.cx, view.cy).detach()
        loss = loss + geometry_loss(out["alpha"], out["normal"], est, out["reg"], 0.05, 0.02)
        loss.backward()
    finally:
        torch.use_deterministic_algorithms(False)
    assert torch.isfinite(res.loss) and abs(float(res.loss) - float(loss)) <= 1e-6 * max(1.0, abs(float(loss)))
    for (name, a), b in zip(auto.param_groups().items(), manual.param_groups().values()):
        ga, gb = a[0].grad, b[0].grad
        if ga is None and gb is None:
            continue
        # the texel gradients are float-atomic sums (order varies run to run); every splat gradient is reproducible
        tol = 1e-5 * float(gb.abs().max()) if name == "texture_dc" else 0.0
        assert float((ga - gb).abs().max()) <= tol, name
    # the geometry terms reach the splats: without them the opacity gradient differs
    plain = GStexTrainer(sc, dev, start_step=3000)
    plain.zero_grad()
    plain.forward_backward(view, gt)
    assert float((plain.opacities.grad - auto.opacities.grad).abs().max()) > 0.0
    # before the switch step both weights are 0 here: the step is the photometric one (no geometry render)
    torch.use_deterministic_algorithms(True)
    try:
        early = GStexTrainer(sc, dev, start_step=2999, lambda_normal=[0.0, 0.05, 3000], lambda_reg=0.0)
        ref = GStexTrainer(sc, dev, start_step=2999)
        for tr in (early, ref):
            tr.zero_grad()
            tr.forward_backward(view, gt)
    finally:
        torch.use_deterministic_algorithms(False)
    assert torch.equal(early.opacities.grad, ref.opacities.grad) and torch.equal(early.means.grad, ref.means.grad)
