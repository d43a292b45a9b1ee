"""GStexTrainer(fused_step=True) (gstex_amd.fused: the photometric training render as one C prologue call and one
autograd node) against the per-op path on the GPU: the prologue's fused kernels compute the per-op outputs with the
same device functions on the same values (gstex_amd/csrc/splat_math.h) and the rest are the same launches, so the
rendered image and the loss are bit-identical, and the gradients agree up to the order of their float-atomic sums; a
few training steps of each path train alike."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(n=4000, texels=80_000, res=96):
    from gstex_amd.scene import make_scene, sphere_view

    dev = torch.device("cuda", 0)
    sc = make_scene(n, texels, seed=5)
    views = [sphere_view(i, res, res).to(dev) for i in range(3)]
    g = torch.Generator().manual_seed(2)
    gts = [torch.rand((res, res, 3), generator=g).to(dev) for _ in range(3)]
    return dev, sc, views, gts


def _count_fused(monkeypatch):
    from gstex_amd import fused

    calls = [0]
    inner = fused.train_render

    def counted(*a, **k):
        calls[0] += 1
        return inner(*a, **k)
    monkeypatch.setattr(fused, "train_render", counted)
    return calls


@pytest.mark.parametrize("n,texels,start", [(4000, 80_000, 3000), (1500, 30_000, 3000), (300, 6_000, 3000),
                                             (4000, 80_000, 1500), (4000, 80_000, 0)])
def test_fused_render_matches_per_op(monkeypatch, n, texels, start):
    """n = 4000: several scan tiles with a partial last one; 1500: one full tile and a partial one; 300: a single
    partial block of the fused preprocessing kernel and a single scan tile.  start 1500: SH degree 1 of the ramp;
    start 0: degree 0, which gstex_train_prologue runs through the per-op entry points."""
    from gstex_amd.model import GStexTrainer

    calls = _count_fused(monkeypatch)
    dev, sc, views, gts = _setup(n, texels)
    tr = GStexTrainer(sc, dev, start_step=start, defer_texture=True, fused_step=True)
    # the first render sizes the pair capacity (one read-back) through the per-op path
    tr.zero_grad()
    tr.forward_backward(views[0], gts[0])
    tr.optimizer_step()
    assert calls[0] == 0 and tr.pairs.capacity > 0
    tr.wait_texture()
    for k in range(3):
        res = {}
        for mode in (True, False):
            tr.fused_step = mode
            tr.zero_grad()
            out = tr.forward_backward(views[k], gts[k])
            torch.cuda.synchronize()
            res[mode] = (out.loss.clone(), out.rgb.clone(),
                         {name: ps[0].grad.detach().clone() for name, ps in tr.param_groups().items()
                          if ps[0].grad is not None})
        assert calls[0] == k + 1
        (lf, rf, gf), (lp, rp, gp) = res[True], res[False]
        assert torch.equal(rf, rp), "fused render differs from the per-op render"
        assert torch.equal(lf, lp)
        assert gf.keys() == gp.keys() and "texture_dc" in gf and "xyz" in gf
        for name in gf:
            a, b = gf[name].double(), gp[name].double()
            scale = max(float(b.abs().max()), 1e-30)
            err = float((a - b).abs().max()) / scale
            assert err < 1e-4, f"{name}: fused gradient differs (max rel {err:.2e})"
            assert float((a - b).abs().mean()) / scale < 1e-7, name
    tr.fused_step = True


def test_fused_step_trains_like_per_op(monkeypatch):
    from gstex_amd.model import LRS, GStexTrainer

    calls = _count_fused(monkeypatch)
    dev, sc, views, gts = _setup()
    a = GStexTrainer(sc, dev, start_step=3000, defer_texture=True, fused_step=False)
    b = GStexTrainer(sc, dev, start_step=3000, defer_texture=True, fused_step=True)
    for step in range(6):
        for tr in (a, b):
            tr.zero_grad()
            tr.forward_backward(views[step % 3], gts[step % 3])
            tr.optimizer_step()
    assert calls[0] == 5  # every step after the capacity-sizing first one
    assert a.skipped_steps == b.skipped_steps == []
    for (name, pa), pb in zip(a.param_groups().items(), b.param_groups().values()):
        x, y = pa[0].detach().double(), pb[0].detach().double()
        if name == "texture_dc":
            x, y = a.texels().double(), b.texels().double()
        scale = max(float(x.abs().max()), 1e-30)
        d = (x - y).abs()
        assert float(d.max()) <= LRS[name] and float(d.mean()) / scale < 1e-6, name


def test_fused_step_with_gradsync_trains_like_per_op(monkeypatch):
    """The fused render under gstex_amd.dist.GradSync (world 1, gloo): the flat buffer's texel slice as the sink, the
    deferred texel update run right before the raster forward once its collective has landed, the head-first exchange
    -- trains like the per-op render under the same GradSync."""
    import socket

    import torch.distributed as dist

    from gstex_amd.dist import GradSync
    from gstex_amd.model import LRS, GStexTrainer

    calls = _count_fused(monkeypatch)
    dev, sc, views, gts = _setup()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        trs = [GStexTrainer(sc, dev, start_step=3000, defer_texture=True, fused_step=f) for f in (False, True)]
        syncs = [GradSync(tr, 1) for tr in trs]
        for step in range(5):
            for tr, sy in zip(trs, syncs):
                sy.zero()
                tr.forward_backward(views[step % 3], gts[step % 3])
                tr.optimizer_step(sync=sy)
        assert calls[0] == 4
        a, b = trs
        for (name, pa), pb in zip(a.param_groups().items(), b.param_groups().values()):
            x, y = pa[0].detach().double(), pb[0].detach().double()
            if name == "texture_dc":
                x, y = a.texels().double(), b.texels().double()
            scale = max(float(x.abs().max()), 1e-30)
            d = (x - y).abs()
            assert float(d.max()) <= LRS[name] and float(d.mean()) / scale < 1e-6, name
    finally:
        if own:
            dist.destroy_process_group()


def test_epilogue_matches_per_op_entry_points():
    """gstex_train_epilogue (setup bwd + activation bwd + SH rest bwd in one kernel) writes bit-identical gradients to
    gstex_raster_setup_bwd_aabb -> gstex_activate_bwd / gstex_sh_rest_bwd on the same accumulator rows."""
    import ctypes

    from gstex_amd import _lib, ops
    from gstex_amd.activations import activate
    from gstex_amd.model import GStexTrainer

    dev, sc, views, _ = _setup(1500, 30_000)
    tr = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
    view = views[1]
    with torch.no_grad():
        qn, scl, op, uv0, umap, vmap, vd = activate(tr.means, tr.quats, tr.scales, tr.opacities, tr.mappings,
                                                    view.campos)
        _, _, _, nth = ops.preprocess(tr.means, scl, 1, qn, view.viewmat, (view.fx, view.fy, view.cx, view.cy),
                                      view.H, view.W)
    n, n_rest = tr.means.shape[0], tr.features_rest.shape[1]
    g = torch.Generator().manual_seed(7)
    partials = (torch.randn((n, 24), generator=g) * 1e-3).to(dev)
    vm, cw = ops._viewmat(view.viewmat), ops._c2w(view.c2w)
    cam = _lib.make_camera(vm, cw, view.fx, view.fy, view.cx, view.cy, view.H, view.W, ops.BLOCK_WIDTH)
    offsets = torch.zeros((n + 1,), device=dev, dtype=torch.int32)
    f = dict(device=dev, dtype=torch.float32)

    def bufs():
        return dict(v_means=torch.empty((n, 3), **f), v_quats=torch.empty((n, 4), **f),
                    v_log_scales=torch.empty((n, 3), **f), v_opac_logits=torch.empty((n, 1), **f),
                    v_rest=torch.empty((n, n_rest, 3), **f), v_sc=torch.empty((n, 3), **f),
                    v_qn=torch.empty((n, 4), **f), v_rgbs=torch.empty((n, 3), **f), v_op=torch.empty((n, 1), **f),
                    v_c=torch.empty((n, 2), **f), v_uv=torch.empty((n, 2), **f))
    P = _lib.ptr
    st = _lib.stream_of(dev)
    a = bufs()
    _lib.call("gstex_raster_setup_bwd_aabb", n, P(tr.means), P(scl), 1.0, P(qn), P(op), P(umap), P(vmap), P(nth),
              P(offsets), P(partials), None, 24, -1, cam, P(a["v_means"]), P(a["v_sc"]), P(a["v_qn"]),
              P(a["v_rgbs"]), P(a["v_op"]), P(a["v_c"]), P(a["v_uv"]), st)
    _lib.call("gstex_sh_rest_bwd", n, 3, n_rest, P(vd), P(a["v_rgbs"]), P(a["v_rest"]), st)
    _lib.call("gstex_activate_bwd", n, P(tr.quats), P(tr.scales), P(op), P(a["v_qn"]), P(a["v_sc"]), P(a["v_op"]),
              P(a["v_quats"]), P(a["v_log_scales"]), P(a["v_opac_logits"]), st)
    b = bufs()
    e = _lib.GstexTrainEpilogueArgs(
        n=n, sh_degree=3, n_rest=n_rest, cam=cam, means=P(tr.means), scales=P(scl), quats_n=P(qn), quats=P(tr.quats),
        log_scales=P(tr.scales), opacities=P(op), umap=P(umap), vmap=P(vmap), viewdirs=P(vd), num_tiles_hit=P(nth),
        offsets=P(offsets), partials=P(partials), v_means=P(b["v_means"]), v_quats=P(b["v_quats"]),
        v_log_scales=P(b["v_log_scales"]), v_opac_logits=P(b["v_opac_logits"]), v_features_rest=P(b["v_rest"]),
        v_scales_act=P(b["v_sc"]), v_quats_n=P(b["v_qn"]), v_rgbs=P(b["v_rgbs"]), v_opacities_act=P(b["v_op"]),
        v_centers=P(b["v_c"]), v_uv0=P(b["v_uv"]))
    _lib.call("gstex_train_epilogue", ctypes.byref(e), st)
    torch.cuda.synchronize()
    assert int((nth > 0).sum()) > n // 2
    for k in ("v_means", "v_quats", "v_log_scales", "v_opac_logits", "v_rest", "v_rgbs"):
        assert torch.equal(a[k], b[k]), k
