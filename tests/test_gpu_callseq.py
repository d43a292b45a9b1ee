"""GPU replay of the reference's own gstex_cuda call sequence.

tests/golden/callseq.{json,npz} hold every call nerfstudio/models/gstex.py:992-1236 (GStexModel.get_outputs) makes
into gstex_cuda in three modes -- training, the eval render (extra_stuff: three 6-channel calls, the last with
settings | 1 << 15) and the viewer's cached path -- recorded with its exact argument structure (positional order, the
int 1 glob_scale, viewmat.squeeze()[:3, :], the non-contiguous c2w = viewmat.inverse(), texture_info, the
background=zeros_like / use_torch_impl=False keywords) and the seeded inputs.  Here each call is made again, in order,
through the real gstex_cuda shim on the GPU, functions resolved from the modules the reference imports them from;
an argument that was an earlier call's output (centres, extents, depths, tile counts, SH colours) is the REPLAYED
output, so the calls chain as in the reference.  Checked against the CPU oracle's answers recorded with the calls:
  * project_points / get_aabb_2d / get_num_tiles_hit_2d bit-exact (xys within 1e-6), spherical_harmonics bit-exact;
  * texture_gaussians: a tuple whose first six entries unpack as gstex.py:1172 does, with the reference's shapes, and
    every output within the parity tolerance of the oracle (tests/helpers.py assert_close_fwd);
  * the images the reference builds from the returned tuples (composite gstex.py:1204-1205; eval: test / uv / edit /
    clean-normal images gstex.py:1183-1203) equal the ones it built from the oracle's outputs, within tolerance;
  * training: the backward of the recorded call for a photometric upstream gradient (img, tex, alpha) vs the oracle's
    fp64 gradients, within max(1e-5, 4 x the oracle's own fp32 error) (the parity tests' criterion).
"""
import numpy as np
import pytest
import torch

from callseq import build, expected_outputs, load, resolve
from helpers import FLIP_MARGIN, GRAD_RTOL, assert_close_fwd, grad_norm_err, grad_rel_err, upstream

pytestmark = pytest.mark.gpu
DEV = "cuda"
NAMES = ("img", "depth", "reg", "alpha", "tex", "normal")
# texture_gaussians positional arguments that carry gradients in the training call -> the oracle's gradient names
GRAD_ARGS = {2: "centers", 6: "rgbs", 7: "opacities", 8: "means", 9: "scales", 11: "quats", 15: "texture"}


@pytest.fixture(scope="module")
def golden():
    return load()


def _replay(meta, arrays, sc, grads=False):
    outs, leaves_by_call, results = [], {}, []
    for i, c in enumerate(meta["scenarios"][sc]["calls"]):
        leaves = []
        train = grads and c["fn"] == "texture_gaussians" and c.get("train_grads", False)
        args = [build(d, arrays, outs, DEV, leaves, train) for d in c["args"]]
        kwargs = {k: build(d, arrays, outs, DEV) for k, d in c["kwargs"].items()}
        r = resolve(c["fn"])(*args, **kwargs)
        outs.append(r if isinstance(r, tuple) else (r,))
        leaves_by_call[i] = (args, leaves)
        results.append(r)
    return outs, leaves_by_call


def _check_preprocessing(meta, arrays, sc, outs):
    for i, c in enumerate(meta["scenarios"][sc]["calls"]):
        exp = expected_outputs(sc, i, c["n_out"], arrays)
        got = [o.detach().cpu() for o in outs[i]]
        if c["fn"] == "project_points":
            assert (got[0] - exp[0]).abs().max().item() <= 1e-6 * max(1.0, exp[0].abs().max().item())
            assert torch.equal(got[1], exp[1]), f"{sc}: depths not bit-exact"
        elif c["fn"] in ("get_aabb_2d", "get_num_tiles_hit_2d", "spherical_harmonics"):
            for g, e in zip(got, exp):
                assert torch.equal(g, e), f"{sc}: {c['fn']} not bit-exact (max {(g.double() - e.double()).abs().max()})"


def _check_raster(meta, arrays, sc, i, c, out):
    H, W = meta["H"], meta["W"]
    C = c["args"][0]["seq"][2]["py"]
    assert isinstance(out, tuple) and len(out) >= 6
    out_img, out_depth, out_reg, out_alpha, out_texture, out_normal = out[:6]  # gstex.py:1172
    assert tuple(out_img.shape) == (H, W, 3) and tuple(out_alpha.shape) == (H, W)
    assert tuple(out_depth.shape) == (H, W) and tuple(out_reg.shape) == (H, W)
    assert tuple(out_texture.shape) == (H, W, C) and tuple(out_normal.shape) == (H, W, 3)
    gpu = {k: o.detach().cpu() for k, o in zip(NAMES, out)}
    ref = {k: torch.from_numpy(arrays[f"{sc}/{i}/o64_{k}"]) for k in NAMES}
    assert_close_fwd(gpu, ref, margin=torch.from_numpy(arrays[f"{sc}/{i}/margin"]))
    return gpu


@pytest.mark.parametrize("sc", ["train", "eval", "viewer"])
def test_reference_call_sequence_replays_through_the_shim(golden, sc):
    meta, arrays = golden
    with torch.no_grad():
        outs, _ = _replay(meta, arrays, sc)
    _check_preprocessing(meta, arrays, sc, outs)
    calls = meta["scenarios"][sc]["calls"]
    rasters = [i for i, c in enumerate(calls) if c["fn"] == "texture_gaussians"]
    gpu = {i: _check_raster(meta, arrays, sc, i, calls[i], outs[i]) for i in rasters}
    # the reference's handling of the returned tuples, restated (gstex.py:1204-1205 and, eval, 1183-1203), against the
    # images the reference itself built from the oracle's answers
    img = {k: torch.from_numpy(v) for k, v in arrays.items() if k.startswith(f"{sc}/images/")}
    bg = img[f"{sc}/images/background"]
    o = gpu[rasters[0]]
    rgb = torch.clamp(o["img"] + o["tex"][:, :, 0:3] + (1 - o["alpha"][:, :, None]) * bg, 0.0, 1.0)
    # pixels with a threshold decision within FLIP_MARGIN of its threshold in any of the calls (an exp ulp may flip it;
    # assert_close_fwd above bounds how many) are left out of the image comparisons
    keep = torch.ones(meta["H"], meta["W"], dtype=torch.bool)
    for i in rasters:
        keep &= ~(torch.from_numpy(arrays[f"{sc}/{i}/margin"]) < FLIP_MARGIN)

    def close(mine, name):
        ref = img[f"{sc}/images/{name}"]
        err = (mine - ref).abs()[keep]
        assert float(err.max()) <= 3e-5, f"{sc} image {name}: max err {float(err.max()):.2e}"

    close(rgb, "rgb")
    if sc == "eval":
        t, n = gpu[rasters[1]], gpu[rasters[2]]
        test_img = t["img"] + (1 - t["alpha"][:, :, None]) * bg
        uv_im = torch.clamp(t["tex"][:, :, 3:6] + (1 - t["alpha"][:, :, None]) * bg, 0.0, 1.0)
        edit = torch.clamp(o["img"] + n["tex"][:, :, :3] + (1 - o["alpha"][:, :, None]) * bg, 0.0, 1.0)
        clean = torch.clamp(0.5 * (n["normal"] + 1) + (1 - o["alpha"][:, :, None]) * bg, 0.0, 1.0)
        for name, mine in (("test", test_img), ("uv", uv_im), ("edit", edit), ("clean_normal_img", clean)):
            close(mine, name)
        # settings | 1 << 15: unit normals where anything was accumulated
        nn = n["normal"].norm(dim=-1)
        hit = o["alpha"] > 1e-3
        assert float((nn[hit] - 1).abs().max()) < 1e-5


def test_reference_training_call_backward(golden):
    """The training call's backward (autograd, engine/trainer.py:460) for the upstream gradient a photometric loss
    sends (img, tex, alpha), through the shim, vs the oracle's fp64 gradients."""
    meta, arrays = golden
    sc = "train"
    outs, leaves_by_call = _replay(meta, arrays, sc, grads=True)
    i = next(k for k, c in enumerate(meta["scenarios"][sc]["calls"]) if c["fn"] == "texture_gaussians")
    args, _ = leaves_by_call[i]
    out = outs[i]
    H, W = meta["H"], meta["W"]
    mask = torch.from_numpy(arrays[f"{sc}/{i}/flip_mask"])
    up = upstream(H, W, 3, 5, mask)
    torch.autograd.backward([out[0], out[3], out[4]], [up["img"].to(DEV), up["alpha"].to(DEV), up["tex"].to(DEV)])
    for k, name in GRAD_ARGS.items():
        t = args[k]
        assert t.requires_grad and t.grad is not None, name
        g = t.grad.detach().cpu()
        g64 = torch.from_numpy(arrays[f"{sc}/{i}/g64_{name}"])
        g32 = torch.from_numpy(arrays[f"{sc}/{i}/g32_{name}"])
        for err_fn in (grad_norm_err, lambda a, b: grad_rel_err(a, b)[0]):
            err, inh = err_fn(g, g64), err_fn(g32, g64)
            assert err <= GRAD_RTOL, f"{name}: rel err {err:.2e} (the oracle's own fp32 error {inh:.2e})"
