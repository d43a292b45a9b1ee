"""HIP path (through the gstex_cuda surface / C-ABI) vs the CPU oracle.  Needs an MI355X.

Tolerances (written here, per north_star): integer/index work bit-exact; forward images within
1e-5 abs + 1e-5 rel of the oracle's fp64 evaluation (same fp32 decisions).  Gradients, against
the oracle's fp64 autograd of the same function:
  * norm-wise relative error ||g - ref|| / ||ref|| and element-wise max|g - ref| / max|ref| are each
    <= 1e-5, outright.  The raster record is evaluated in fp64 and rounded once (raster.hip setup_kernel;
    setup_bwd_chain in fp64), and near-edge-on splats (|normal . view dir| < 0.1, whose p = dx A + dy B + (0, 0, Pz)
    is a small difference of larger terms) take p from their fp64 setup row in the forward and the backward alike
    (DESIGN.md §4); the oracle restates both (RasterInputs.hp) and evaluates with the fp32-rounded camera
    intrinsics the kernels receive.  The oracle's own fp32 autograd error is printed beside each result (it is
    the yardstick, no longer part of the bound).  Measured (profiles/r06_parity_hp.log): every gradient of every
    case <= 8.8e-6 norm-wise and <= 4.6e-6 max-element (cfg3 96x96: means / quats 3.0e-6 / 3.3e-6 norm-wise).
"""
import numpy as np
import pytest
import torch

from helpers import DIFF, GRAD_RTOL, assert_close_fwd, gpu_run, grad_norm_err, grad_rel_err, make_case, \
    oracle_run, upstream
from oracle import raster as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _report(tag, d):
    print(f"[parity] {tag}: " + ", ".join(f"{k}={v:.2e}" for k, v in d.items()))


# ---------------------------------------------------------------- preprocessing
def test_project_points_and_aabb_match_oracle():
    import gstex_cuda

    case = make_case(n=2000, n_texels=0, H=100, W=120, seed=3, cube=3.0)
    v = case.view
    inp = case.inp
    intr = (v.fx, v.fy, v.cx, v.cy)
    xys, depths = gstex_cuda.project_points(inp.means.to(DEV), v.viewmat.to(DEV), intr)
    cam = inp.cam
    oxy, odep = O.project_points(inp.means, cam)
    assert torch.equal(depths.cpu(), odep), "depths not bit-exact"
    assert (xys.cpu() - oxy).abs().max().item() <= 1e-6 * max(1.0, oxy.abs().max().item())
    c, e = gstex_cuda.get_aabb_2d(inp.means.to(DEV), inp.scales.to(DEV), 1, inp.quats.to(DEV), v.viewmat.to(DEV), intr)
    oc, oe = O.aabb_2d(inp.means, inp.scales, 1.0, inp.quats, cam)
    assert torch.equal(c.cpu(), oc.detach()), f"centers not bit-exact: {(c.cpu() - oc).abs().max()}"
    assert torch.equal(e.cpu(), oe), f"extents not bit-exact: {(e.cpu() - oe).abs().max()}"
    nth = gstex_cuda.get_num_tiles_hit_2d(c, e, 100, 120, 16)
    onth = O.num_tiles_hit(oc, oe, 100, 120)
    assert torch.equal(nth.cpu(), onth)
    assert int((nth == 0).sum()) > 0, "case should contain culled / off-screen splats"
    # the fused launch (gstex_preprocess, the training path): the same three outputs, bit for bit
    from gstex_amd import ops

    d2, c2, e2, n2 = ops.preprocess(inp.means.to(DEV), inp.scales.to(DEV), 1, inp.quats.to(DEV), v.viewmat.to(DEV),
                                    intr, 100, 120)
    assert torch.equal(d2.cpu(), odep) and torch.equal(c2, c) and torch.equal(e2, e) and torch.equal(n2, nth)


def test_aabb_and_projection_backward():
    import gstex_cuda

    case = make_case(n=500, n_texels=0, H=64, W=64, seed=4)
    v, inp, cam = case.view, case.inp, case.inp.cam
    intr = (v.fx, v.fy, v.cx, v.cy)
    g = torch.Generator().manual_seed(1)
    vc = torch.randn(500, 2, generator=g)
    leaves = [inp.means.to(DEV).requires_grad_(True), inp.scales.to(DEV).requires_grad_(True),
              inp.quats.to(DEV).requires_grad_(True)]
    c, _ = gstex_cuda.get_aabb_2d(leaves[0], leaves[1], 1, leaves[2], v.viewmat.to(DEV), intr)
    (c * vc.to(DEV)).sum().backward()
    ol = [inp.means.double().requires_grad_(True), inp.scales.double().requires_grad_(True),
          inp.quats.double().requires_grad_(True)]
    oc, _ = O.aabb_2d(ol[0], ol[1], 1.0, ol[2], cam, dtype=torch.float64)
    (oc * vc.double()).sum().backward()
    errs = {}
    for name, a, b in zip(["means", "scales", "quats"], leaves, ol):
        errs[name], _ = grad_rel_err(a.grad.cpu(), b.grad)
    _report("aabb_bwd", errs)
    assert max(errs.values()) < 1e-4
    # projection backward
    m = inp.means.to(DEV).requires_grad_(True)
    xy, dep = gstex_cuda.project_points(m, v.viewmat.to(DEV), intr)
    (xy * vc.to(DEV)).sum().add((dep * vc[:, 0].to(DEV)).sum()).backward()
    om = inp.means.double().requires_grad_(True)
    oxy, odep = O.project_points(om, cam, dtype=torch.float64)
    (oxy * vc.double()).sum().add((odep * vc[:, 0].double()).sum()).backward()
    e, _ = grad_rel_err(m.grad.cpu(), om.grad)
    _report("project_bwd", {"means": e})
    assert e < 1e-5


# ---------------------------------------------------------------- binning
def _bins_equal(case):
    from gstex_amd.ops import bin_and_sort

    inp = case.inp
    H, W = inp.cam.H, inp.cam.W
    off, tr, ids, slots = bin_and_sort(inp.centers.to(DEV), inp.extents.to(DEV), inp.depths.to(DEV),
                                       case.nth.to(DEV), H, W, 16)
    o_off, o_tr, o_ids, o_slots = O.bin_and_sort(inp.centers, inp.extents, inp.depths, H, W)
    assert np.array_equal(off.cpu().numpy(), o_off)
    assert np.array_equal(tr.cpu().numpy(), o_tr)
    assert np.array_equal(ids.cpu().numpy(), o_ids)
    assert np.array_equal(slots.cpu().numpy(), o_slots)
    return o_tr


def test_binning_bit_exact():
    case = make_case(n=3000, n_texels=0, H=96, W=112, seed=5)
    tr = _bins_equal(case)
    assert (tr[:, 1] - tr[:, 0]).max() > 0


def test_binning_many_tiles_global_count_path():
    # > 16384 tiles: the LDS-privatised tile histogram does not fit, counting falls back to global atomics
    case = make_case(n=1500, n_texels=0, H=2080, W=2080, seed=8)
    tr = _bins_equal(case)
    assert tr.shape[0] > 16384 and (tr[:, 1] - tr[:, 0]).max() > 0


def test_binning_large_bucket_merge_path():
    # many splats piled on few tiles -> buckets > 4096 keys exercise the merge-path sort
    case = make_case(n=20000, n_texels=0, H=32, W=32, seed=6, cube=0.3)
    tr = _bins_equal(case)
    assert (tr[:, 1] - tr[:, 0]).max() > 4096 * 2


@pytest.mark.parametrize("n", [200, 450, 1000, 2000, 4000])
def test_binning_register_sort_sizes(n):
    # every splat on the same 4 tiles: buckets of ~n keys exercise each register-sort width (256 E keys, E = 1..16)
    case = make_case(n=n, n_texels=0, H=32, W=32, seed=9, cube=0.3)
    tr = _bins_equal(case)
    assert 0 < (tr[:, 1] - tr[:, 0]).max() <= 4096


def test_binning_equal_depths_tie_break():
    case = make_case(n=400, n_texels=0, H=48, W=48, seed=7)
    case.inp.depths = torch.full_like(case.inp.depths, 3.0)  # every key ties on depth -> id order
    _bins_equal(case)


# ---------------------------------------------------------------- raster forward / backward
CASES = {
    "tex3_default": dict(n=300, n_texels=20000, H=64, W=80, seed=0),
    "tex6_eval": dict(n=250, n_texels=15000, H=48, W=64, seed=1, C=6, settings=(1 << 9) | (1 << 10) | (1 << 15)),
    "tex1_generic": dict(n=200, n_texels=8000, H=40, W=40, seed=2, C=1),
    "no_aa": dict(n=300, n_texels=20000, H=64, W=64, seed=3, settings=1 << 10),
    "no_reg": dict(n=300, n_texels=20000, H=64, W=64, seed=4, settings=1 << 9),
    "settings0": dict(n=300, n_texels=20000, H=64, W=64, seed=5, settings=0),
    "2dgs_T0": dict(n=400, n_texels=0, H=56, W=72, seed=6),
    "opaque": dict(n=300, n_texels=20000, H=64, W=64, seed=7, opacity=0.98),
    "background": dict(n=200, n_texels=10000, H=50, W=70, seed=8, bg=(0.2, 0.5, 0.9)),
    "ragged_17x33": dict(n=150, n_texels=5000, H=17, W=33, seed=9),
    # ~1000 texels per splat: 16-splat batches overflow the LDS staging -> global-atomic texel path
    "big_texel_blocks": dict(n=60, n_texels=60000, H=64, W=64, seed=10),
}


@pytest.mark.parametrize("name", list(CASES))
def test_raster_forward_backward(name):
    _check_raster(name, None)


# img / alpha / tex gradients only (depth, distortion and normal gradients None, the training default):
# the backward runs its specialisation without those terms
@pytest.mark.parametrize("name", ["tex3_default", "tex6_eval", "no_aa", "ragged_17x33", "big_texel_blocks"])
def test_raster_backward_photometric_only(name):
    _check_raster(name, ("img", "alpha", "tex"))


def _check_raster(name, outputs):
    case = make_case(**CASES[name])
    o32, o64, aux, og = oracle_run(case, grads=True, outputs=outputs)
    gout, gg = gpu_run(case, grads=True, outputs=outputs)
    fwd = {k: (gout[k].double() - o64[k]).abs().max().item() for k in gout}
    _report(f"{name} fwd", fwd)
    assert_close_fwd(gout, o64, margin=aux["margin"])
    _, _, _, og32 = oracle_run(case, grads=True, grad_dtype=torch.float32, outputs=outputs)
    errs, norm_errs, inherent, inherent_n = {}, {}, {}, {}
    for k in DIFF:
        errs[k], _ = grad_rel_err(gg[k], og[k])
        inherent[k], _ = grad_rel_err(og32[k], og[k])
        norm_errs[k] = grad_norm_err(gg[k], og[k])
        inherent_n[k] = grad_norm_err(og32[k], og[k])
    _report(f"{name} bwd max-rel", errs)
    _report(f"{name} bwd fp32-oracle max-rel", inherent)
    _report(f"{name} bwd norm-rel", norm_errs)
    for k in DIFF:
        assert norm_errs[k] <= GRAD_RTOL, f"{name}: grad {k} norm-wise rel err {norm_errs[k]:.3e} > {GRAD_RTOL:.0e}"
        assert errs[k] <= GRAD_RTOL, f"{name}: grad {k} max rel err {errs[k]:.3e} > {GRAD_RTOL:.0e}"


def test_raster_without_near_edge_on_rows(monkeypatch):
    """GSTEX_HP=0 (no hp_records buffer: the marks are ignored, every pair evaluated from the fp32 record) against the
    oracle restating that path (RasterInputs.hp = False): the forward within the usual tolerance; the gradients
    within 1e-4 (the fp32 record's conditioning, DESIGN.md §4, is what the rows remove)."""
    from gstex_amd import ops

    monkeypatch.setattr(ops, "HP_RECORDS", False)
    case = make_case(**CASES["no_reg"])
    case.inp.hp = False
    o32, o64, aux, og = oracle_run(case, grads=True)
    gout, gg = gpu_run(case, grads=True)
    assert_close_fwd(gout, o64, margin=aux["margin"])
    errs = {k: grad_norm_err(gg[k], og[k]) for k in DIFF}
    _report("no hp rows bwd norm-rel", errs)
    for k, e in errs.items():
        assert e <= 1e-4, f"grad {k} norm-wise rel err {e:.3e}"


def test_empty_and_offscreen():
    case = make_case(n=50, n_texels=1000, H=32, W=32, seed=10)
    case.nth = torch.zeros_like(case.nth)  # nothing visible
    case.inp.extents = torch.zeros_like(case.inp.extents)
    gout, gg = gpu_run(case, grads=True)
    assert torch.all(gout["alpha"] == 0) and torch.all(gout["img"] == 0)
    for k in DIFF:
        assert torch.all(gg[k] == 0), k


def test_backward_is_deterministic(deterministic):
    case = make_case(n=300, n_texels=20000, H=64, W=64, seed=11)
    _, g1 = gpu_run(case, grads=True)
    _, g2 = gpu_run(case, grads=True)
    for k in ["rgbs", "opacities", "means", "scales", "quats", "centers"]:
        assert torch.equal(g1[k], g2[k]), f"{k} gradient not bitwise reproducible"


@pytest.mark.parametrize("geo", [False, True])
def test_atomic_splat_sums_match_rows(geo):
    """Default mode (per-splat float-atomic accumulators, no rows, no summing pass) against the deterministic
    per-pair rows: the same sums up to summation order, for 24-value (photometric) and 32-value rows."""
    case = make_case(n=700, n_texels=30000, H=80, W=96, seed=29)
    outs = None if geo else ("img", "alpha", "tex")
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        _, g_rows = gpu_run(case, grads=True, outputs=outs)
    finally:
        torch.use_deterministic_algorithms(False)
    _, g_atom = gpu_run(case, grads=True, outputs=outs)
    for k in ["rgbs", "opacities", "means", "scales", "quats", "centers", "uv0", "texture"]:
        assert grad_norm_err(g_atom[k], g_rows[k]) < 1e-6, k
        assert float(g_rows[k].abs().max()) > 0, k



# ---------------------------------------------------------------- launch order (scheduling only)
@pytest.mark.parametrize("n_tiles", [1, 2500, 16384, 16385])
def test_tile_order_is_largest_first(n_tiles):
    from gstex_amd.ops import tile_order

    g = np.random.default_rng(n_tiles)
    counts = g.integers(0, 40, n_tiles)
    counts[g.integers(0, n_tiles, max(1, n_tiles // 50))] = 1 << 19  # beyond the 2^18-1 clamp: ties
    ends = np.cumsum(counts)
    tr = np.stack([ends - counts, ends], 1).astype(np.int64)
    tr = np.clip(tr, 0, 2**31 - 1).astype(np.int32)
    got = tile_order(torch.from_numpy(tr).to(DEV)).cpu().numpy()
    if n_tiles > 16384:
        assert np.array_equal(got, np.arange(n_tiles)), "above 16384 tiles the order is row-major"
        return
    cnt = np.minimum(tr[:, 1] - tr[:, 0], (1 << 18) - 1)
    expect = np.lexsort((np.arange(n_tiles), -cnt))
    assert np.array_equal(got, expect)


@pytest.mark.parametrize("n_units,groups", [(1, 1), (10000, 8), (200003, 8), (40000, 1)])
def test_unit_order(n_units, groups):
    """gstex_unit_order: units of cost 0 take no position; the others by descending cost inside their XCD group,
    the k-th of group g at position 8 k + g -- or, with groups too uneven (a single group here), by descending cost
    overall."""
    from gstex_amd.ops import unit_order

    g = np.random.default_rng(n_units)
    cost = g.integers(0, 300, n_units).astype(np.int64)
    cost[g.integers(0, n_units, max(1, n_units // 50))] = 1 << 17  # beyond the 1023 clamp
    grp = g.integers(0, groups, n_units)
    key = (cost | (grp << 24)).astype(np.int32)
    got = unit_order(torch.from_numpy(key).to(DEV)).cpu().numpy()
    placed = got[got >= 0]
    assert np.array_equal(np.sort(placed), np.nonzero(cost > 0)[0]), "every non-empty unit exactly once"
    c = np.minimum(cost, 1023)
    counts = np.bincount(grp[cost > 0], minlength=8)
    if 8 * counts.max() <= n_units:
        pos = np.nonzero(got >= 0)[0]
        assert np.all(grp[got[pos]] == pos % 8), "unit not at a position of its group"
        for r in range(8):
            seq = got[r::8]
            seq = seq[seq >= 0]
            assert np.all(np.diff(c[seq]) <= 0)
    else:
        assert np.all(got[:len(placed)] >= 0) and np.all(np.diff(c[placed]) <= 0)


@pytest.mark.parametrize("H,W,n", [(80, 96, 400), (64, 64, 0), (2064, 2064, 3000)])  # 16641 tiles: row-major
def test_bin_sort_ordered_matches_tile_order(H, W, n):
    """gstex_bin_sort_ordered: the binning as gstex_bin_sort, plus the launch order gstex_tile_order computes
    from the resulting tile ranges (the forward reuses it instead of ranking the tiles twice)."""
    from gstex_amd import ops

    g = torch.Generator().manual_seed(n + H)
    centers = (torch.rand((n, 2), generator=g) * torch.tensor([W, H])).to(DEV)
    extents = (torch.rand((n, 2), generator=g) * 40 + 1).to(DEV)
    depths = (torch.rand((n,), generator=g) + 0.5).to(DEV)
    nth = ops.get_num_tiles_hit_2d(centers, extents, H, W, 16)
    a = ops.bin_and_sort(centers, extents, depths, nth, H, W)
    b = ops.bin_finish(ops.bin_begin(nth), centers, extents, depths, H, W, with_order=True)
    for x, y in zip(a, b[:4]):
        assert torch.equal(x, y)
    assert torch.equal(b[4], ops.tile_order(b[1]))


def test_outputs_independent_of_launch_order(monkeypatch, deterministic):
    from gstex_amd import ops

    case = make_case(n=400, n_texels=20000, H=80, W=96, seed=13)
    f1, g1 = gpu_run(case, grads=True)
    finish = ops.bin_finish

    def reversed_order(*a, **k):  # the forward takes its launch order from the binning: reverse it
        out = finish(*a, **k)
        return out[:4] + (out[4].flip(0).contiguous(),) if k.get("with_order") else out

    monkeypatch.setattr(ops, "bin_finish", reversed_order)
    f2, g2 = gpu_run(case, grads=True)
    for k in f1:
        assert torch.equal(f1[k], f2[k]), k
    for k in ["rgbs", "opacities", "means", "scales", "quats", "centers", "uv0"]:
        assert torch.equal(g1[k], g2[k]), k
    # texel gradients sum over tiles with float atomics: equal up to summation order
    t1, t2 = g1["texture"].double(), g2["texture"].double()
    assert float((t1 - t2).abs().max()) <= 1e-6 * float(t1.abs().max())


# ---------------------------------------------------------------- SH / texture_sample
@pytest.mark.parametrize("K", [25, 30])  # LDS-staged kernels up to K = 25, direct kernels above
@pytest.mark.parametrize("degree", [0, 1, 2, 3, 4])
def test_sh_parity(degree, K):
    import gstex_cuda

    g = torch.Generator().manual_seed(degree)
    n = 1000
    dirs = torch.randn(n, 3, generator=g)
    coeffs = torch.randn(n, K, 3, generator=g)
    c = coeffs.to(DEV).requires_grad_(True)
    out = gstex_cuda.spherical_harmonics(degree, dirs.to(DEV), c)
    ref = O.spherical_harmonics(degree, dirs, coeffs)
    assert torch.equal(out.detach().cpu(), ref), "SH forward not bit-exact"
    vo = torch.randn(n, 3, generator=g)
    out.backward(vo.to(DEV))
    oc = coeffs.clone().requires_grad_(True)
    O.spherical_harmonics(degree, dirs, oc).backward(vo)
    assert torch.equal(c.grad.cpu(), oc.grad), "SH backward not bit-exact vs the fp32 oracle"


def test_texture_sample_parity():
    import gstex_cuda
    from gstex_amd.charts import build_charts, texture_dims_to_query

    g = torch.Generator().manual_seed(3)
    log_scales = torch.log(10 ** (-2.5 + 1.5 * torch.rand((400, 3), generator=g)))
    old_dims, _, _ = build_charts(log_scales, 8000)
    new_dims, _, _ = build_charts(log_scales, 12000)
    T = int((old_dims[:, 0] * old_dims[:, 1]).sum())
    tex = torch.rand(T, 3, generator=g)
    ids, uv = texture_dims_to_query(new_dims)
    qd = old_dims[ids].contiguous()
    t = tex.to(DEV).requires_grad_(True)
    out = gstex_cuda.texture_sample((1, 1, 3), qd.to(DEV), t, uv.to(DEV))
    ref = O.texture_sample(qd, tex, uv)
    assert (out.detach().cpu() - ref).abs().max().item() <= 1e-6
    vo = torch.randn(out.shape, generator=g)
    out.backward(vo.to(DEV))
    ot = tex.double().requires_grad_(True)
    O.texture_sample(qd, ot, uv, dtype=torch.float64).backward(vo.double())
    assert (t.grad.cpu().double() - ot.grad).abs().max().item() <= 1e-5
    # the reference-API torch sampler agrees with the HIP sampler
    from gstex_cuda._torch_impl import sample_texture

    assert (sample_texture(qd.to(DEV), tex.to(DEV), uv.to(DEV)).cpu() - ref).abs().max().item() <= 1e-6


# ---------------------------------------------------------------- fused Adam (train-step support)
def test_fused_adam_matches_torch_adam():
    from gstex_amd.optim import FusedAdam

    g = torch.Generator().manual_seed(21)
    shapes = [(200_003, 3), (1000, 1), (7,), (3, 15, 3), (5000, 4), (1,), (33, 1, 2)]
    lrs = [8e-5, 2.5e-3, 1.25e-4, 5e-2, 5e-3, 1e-3, 1e-3]
    base = [torch.randn(s, generator=g) for s in shapes]
    a = [torch.nn.Parameter(t.clone().to(DEV)) for t in base]
    b = [torch.nn.Parameter(t.clone().to(DEV)) for t in base]
    opt_a = FusedAdam([{"params": [p], "lr": lr} for p, lr in zip(a, lrs)], eps=1e-15)
    opt_b = torch.optim.Adam([{"params": [p], "lr": lr} for p, lr in zip(b, lrs)], eps=1e-15, foreach=True)
    for step in range(6):
        for pa, pb in zip(a, b):
            gr = (torch.randn(pa.shape, generator=g) * 10 ** (step % 3 - 2)).to(DEV)
            pa.grad = gr.clone()
            pb.grad = gr.clone()
        if step == 3:  # moments reset mid-run (the rechart): that tensor restarts at t = 1
            opt_a.state.pop(a[0])
            opt_b.state.pop(b[0])
        opt_a.step()
        opt_b.step()
        for pa, pb in zip(a, b):
            # torch's foreach kernels may contract a*b+c into FMAs: equal to within a few ulp
            torch.testing.assert_close(pa.detach(), pb.detach(), rtol=2e-6, atol=1e-7)
    for pa, pb in zip(a, b):
        torch.testing.assert_close(opt_a.state[pa]["exp_avg_sq"], opt_b.state[pb]["exp_avg_sq"], rtol=1e-5, atol=0)


def test_fused_adam_grad_scale_bit_identical():
    """grad_scale (gstex_adam_step_scaled, the data-parallel 1 / world folded into the update) == scaling the gradient
    first and stepping unscaled, bit for bit; with zero_grad the gradient is left zeroed."""
    from gstex_amd.optim import FusedAdam

    g = torch.Generator().manual_seed(22)
    shapes = [(100_001, 3), (513,), (64, 4)]
    base = [torch.randn(s, generator=g) for s in shapes]
    for scale in (0.5, 1.0 / 3.0, 0.125):
        a = [torch.nn.Parameter(t.clone().to(DEV)) for t in base]
        b = [torch.nn.Parameter(t.clone().to(DEV)) for t in base]
        opt_a = FusedAdam([{"params": a, "lr": 1e-3}], eps=1e-15)
        opt_b = FusedAdam([{"params": b, "lr": 1e-3}], eps=1e-15)
        for step in range(3):
            for pa, pb in zip(a, b):
                gr = torch.randn(pa.shape, generator=g).to(DEV)
                pa.grad = gr.clone()
                pb.grad = gr * scale
            opt_a.step(grad_scale=scale, zero_grad=step == 2)
            opt_b.step()
            for pa, pb in zip(a, b):
                assert torch.equal(pa.detach(), pb.detach())
        assert all(float(pa.grad.abs().max()) == 0.0 for pa in a)


# ---------------------------------------------------------------- fused photometric loss (train-step support)
@pytest.mark.parametrize("C", [3, 4])
def test_fused_loss_matches_eager_torch(C):
    from gstex_amd.loss import photometric_loss
    from gstex_amd.model import ssim

    g = torch.Generator().manual_seed(40 + C)
    H, W = 70, 93
    img = (torch.rand(H, W, 3, generator=g) * 1.4 - 0.2)
    tex = torch.rand(H, W, C, generator=g) * 0.3
    alpha = torch.rand(H, W, generator=g)
    bg = torch.rand(3, generator=g)
    gt = torch.rand(H, W, 3, generator=g)
    gt[:5, :5] = 1.0  # with img saturated there too: |gt - rgb| = 0 ties (sign 0)
    img[:5, :5] = 2.0
    leaves = [t.to(DEV).requires_grad_(True) for t in (img, tex, alpha)]
    loss, rgb = photometric_loss(leaves[0], leaves[1], leaves[2], bg.to(DEV), gt.to(DEV))
    loss.backward(torch.tensor(1.7, device=DEV))
    ref_leaves = [t.to(DEV).requires_grad_(True) for t in (img, tex, alpha)]
    r_img, r_tex, r_alpha = ref_leaves
    ref_rgb = torch.clamp(r_img + r_tex[:, :, 0:3] + (1 - r_alpha[:, :, None]) * bg.to(DEV)[None, None, :], 0.0, 1.0)
    gtd = gt.to(DEV)
    ref = 0.8 * torch.abs(gtd - ref_rgb).mean() + 0.2 * (1 - ssim(gtd.permute(2, 0, 1)[None],
                                                               ref_rgb.permute(2, 0, 1)[None]))
    ref.backward(torch.tensor(1.7, device=DEV))
    assert torch.equal(rgb, ref_rgb.detach()), "composite must match the eager expression bit for bit"
    assert abs(float(loss.detach()) - float(ref.detach())) <= 2e-6 * abs(float(ref.detach()))
    for a, b, name in zip(leaves, ref_leaves, ("img", "tex", "alpha")):
        err = float((a.grad - b.grad).abs().max())
        scale = float(b.grad.abs().max())
        assert err <= 1e-5 * scale, f"{name}: max err {err:.3e} vs scale {scale:.3e}"
    assert float(leaves[1].grad[:, :, 3:].abs().sum()) == 0.0


# ---------------------------------------------------------------- texture_edit (viewer paint tool, §8f-4)
@pytest.mark.parametrize("seed", [31, 32])
def test_texture_edit_matches_oracle(seed):
    import gstex_cuda

    case = make_case(n=400, n_texels=30000, H=64, W=80, seed=seed, settings=1 << 13)
    inp, v = case.inp, case.view
    H, W = inp.cam.H, inp.cam.W
    g = torch.Generator().manual_seed(seed)
    rgb = torch.rand(H, W, 3, generator=g)
    a = (torch.rand(H, W, generator=g) > 0.3).float() * torch.rand(H, W, generator=g)
    depth = O.rasterize(inp)[0]["depth"]  # the caller's depth render (gstex.py:572-574)
    dlo, dhi = depth - 1e-2, depth + 1e-2
    ref = O.texture_edit(inp, rgb, a, dlo, dhi)
    dv = lambda t: t.detach().to(DEV).contiguous()  # noqa: E731
    n = inp.means.shape[0]
    out = gstex_cuda.texture_edit(
        (n, 1, 5), dv(inp.texture_dims), dv(rgb), dv(a[..., None]), dv(dlo), dv(dhi), dv(inp.centers),
        dv(inp.extents), dv(inp.depths), dv(case.nth), dv(inp.opacities), dv(inp.means), dv(inp.scales), 1.0,
        dv(inp.quats), dv(inp.uv0), dv(inp.umap), dv(inp.vmap), dv(v.viewmat), dv(v.c2w), v.fx, v.fy, v.cx, v.cy,
        H, W, 16, 1 << 13, background=torch.zeros(3, device=DEV))
    got = out.double().cpu()
    assert got.shape == ref.shape
    assert float(ref[:, 4].sum()) > 1.0, "the stroke must reach texels"
    touched_ref, touched = ref[:, 4] > 0, got[:, 4] > 0
    assert torch.equal(touched_ref, touched), "the same texels are painted (integer decisions)"
    err = (got - ref).abs().max(0).values
    scale = ref.abs().max(0).values
    assert bool((err <= 1e-5 * scale + 1e-9).all()), (err, scale)  # float atomics: summation order only


# ---------------------------------------------------------------- texel affine (SH2RGB on read)
def test_texture_transform_equals_materialised_sh2rgb():
    from gstex_amd import ops

    case = make_case(n=400, n_texels=30000, H=64, W=80, seed=17)
    inp, v = case.inp, case.view
    C0 = 0.28209479177387814
    g = torch.Generator().manual_seed(3)
    dc = torch.randn(inp.texture.shape, generator=g)
    dv = lambda t: t.detach().to(DEV).contiguous()  # noqa: E731
    n = inp.means.shape[0]

    def run(tex_leaf, transform):
        args = ((n, 1, 3), dv(inp.texture_dims), dv(inp.centers), dv(inp.extents), dv(inp.depths), dv(case.nth),
                dv(inp.rgbs), dv(inp.opacities), dv(inp.means), dv(inp.scales), 1.0, dv(inp.quats), dv(inp.uv0),
                dv(inp.umap), dv(inp.vmap))
        outs = ops.texture_gaussians(*args, tex_leaf, dv(v.viewmat), dv(v.c2w), v.fx, v.fy, v.cx, v.cy,
                                     inp.cam.H, inp.cam.W, 16, inp.settings, texture_transform=transform)
        up = upstream(inp.cam.H, inp.cam.W, 3, 5)
        names = ["img", "depth", "reg", "alpha", "tex", "normal"]
        torch.autograd.backward(list(outs), [up[k].to(DEV) for k in names])
        return [o.detach().cpu() for o in outs]

    leaf_dc = dv(dc).requires_grad_(True)
    o1 = run(leaf_dc, (C0, 0.5))
    leaf_tex = (dv(dc) * C0 + 0.5).detach().requires_grad_(True)  # charts.SH2RGB, materialised
    o2 = run(leaf_tex, None)
    for a, b in zip(o1, o2):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-6)
    gd, gt = leaf_dc.grad.double().cpu(), leaf_tex.grad.double().cpu() * C0
    # the two runs stage texel gradients at different fixed-point scales (tex_scale C0 vs 1): each is exact to
    # 2^-25 of its wave's largest upstream texel gradient, so they agree to a few 1e-6 (parity bound: 1e-5)
    assert float((gd - gt).norm() / gt.norm()) < 4e-6


@pytest.mark.parametrize("gscale", [1e-20, 1e12])
def test_texel_fixed_point_scale_invariance(gscale):
    # the backward's per-wave fixed-point scale follows the upstream texel-gradient magnitude: scaling dL/dtex by
    # any factor scales v_texture by the same factor, to the staging resolution (2^-25 of the wave's largest
    # upstream texel gradient; a factor that is not a power of two moves the rounding grid)
    case = make_case(n=300, n_texels=20000, H=64, W=80, seed=12)
    import helpers

    orig = helpers.upstream

    def scaled(H, W, C, seed=5, mask=None):
        up = orig(H, W, C, seed, mask)
        up = {k: torch.zeros_like(v) for k, v in up.items()} | {"tex": up["tex"] * gscale}
        return up

    def unit(H, W, C, seed=5, mask=None):
        up = orig(H, W, C, seed, mask)
        return {k: torch.zeros_like(v) for k, v in up.items()} | {"tex": up["tex"]}

    try:
        helpers.upstream = unit
        _, gu = gpu_run(case, grads=True, seed=5)
        helpers.upstream = scaled
        _, gs = gpu_run(case, grads=True, seed=5)
    finally:
        helpers.upstream = orig
    a, b = gs["texture"].double() / gscale, gu["texture"].double()
    assert float(b.abs().max()) > 0
    assert float((a - b).norm() / b.norm()) < 4e-6


# ---------------------------------------------------------------- fused activations / SH without the DC cat
def test_sh_rest_equals_sh_on_concatenated_coeffs():
    import gstex_cuda
    from gstex_amd.activations import sh_rest

    g = torch.Generator().manual_seed(4)
    n = 3000
    dirs = torch.randn(n, 3, generator=g).to(DEV)
    rest = torch.randn(n, 15, 3, generator=g).to(DEV)
    a = rest.clone().requires_grad_(True)
    b = rest.clone().requires_grad_(True)
    for deg in (1, 3):
        out_a = sh_rest(deg, dirs, a)
        out_b = gstex_cuda.spherical_harmonics(deg, dirs, torch.cat([torch.zeros_like(b[:, :1]), b], 1))
        assert torch.equal(out_a, out_b)
        vo = torch.randn(n, 3, generator=g).to(DEV)
        ga, = torch.autograd.grad(out_a, a, vo)
        gb, = torch.autograd.grad(out_b, b, vo)
        assert torch.equal(ga, gb)


def test_fused_activations_match_eager_trainer():
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    sc = make_scene(3000, 60000, seed=2)
    v = sphere_view(1, 96, 128).to(DEV)
    gt = torch.rand(96, 128, 3, generator=torch.Generator().manual_seed(0)).to(DEV)
    tf = GStexTrainer(sc, DEV, fused_activations=True)
    te = GStexTrainer(sc, DEV, fused_activations=False)
    of, oe = tf.forward_backward(v, gt), te.forward_backward(v, gt)
    assert abs(float(of.loss) - float(oe.loss)) <= 1e-5 * abs(float(oe.loss))
    assert float((of.rgb - oe.rgb).abs().max()) < 1e-4
    for pf, pe, name in zip(tf.parameters(), te.parameters(), ["means", "features_dc", "features_rest", "opacities",
                                                                "scales", "quats", "texture_dc"]):
        if pe.grad is None:
            assert pf.grad is None or float(pf.grad.abs().max()) == 0.0, name
            continue
        err = float((pf.grad - pe.grad).norm() / pe.grad.norm().clamp(min=1e-30))
        assert err < 1e-4, f"{name}: rel err {err:.2e}"


# ---------------------------------------------------------------- folded AABB-centre chain (training path)
def test_fold_aabb_gradients_bit_identical(deterministic):
    """texture_gaussians(fold_aabb=True) chains the centre gradient through get_aabb_2d inside the raster's
    setup backward: means / scales / quats gradients are bit-identical to the separate get_aabb_2d backward
    plus autograd's accumulation."""
    import gstex_cuda

    case = make_case(n=600, n_texels=30000, H=72, W=88, seed=21)
    v, inp = case.view, case.inp
    intr = (v.fx, v.fy, v.cx, v.cy)
    dv = lambda t: t.detach().to(DEV).contiguous()  # noqa: E731
    up = upstream(inp.cam.H, inp.cam.W, case.C, 8)
    res = []
    for fold in (False, True):
        leaves = {k: dv(getattr(inp, k)).requires_grad_(True) for k in ("means", "scales", "quats", "rgbs",
                                                                          "opacities", "texture", "uv0")}
        c, e = gstex_cuda.get_aabb_2d(leaves["means"], leaves["scales"], inp.glob_scale, leaves["quats"],
                                      dv(v.viewmat), intr)
        _, depths = gstex_cuda.project_points(leaves["means"], dv(v.viewmat), intr)
        nth = gstex_cuda.get_num_tiles_hit_2d(c, e, inp.cam.H, inp.cam.W, 16)
        outs = gstex_cuda.texture_gaussians(
            (inp.means.shape[0], 1, case.C), dv(inp.texture_dims), c, e, depths, nth, leaves["rgbs"],
            leaves["opacities"], leaves["means"], leaves["scales"], inp.glob_scale, leaves["quats"], leaves["uv0"],
            dv(inp.umap), dv(inp.vmap), leaves["texture"], dv(v.viewmat), dv(v.c2w), v.fx, v.fy, v.cx, v.cy,
            inp.cam.H, inp.cam.W, 16, inp.settings, fold_aabb=fold)
        names = ["img", "depth", "reg", "alpha", "tex", "normal"]
        torch.autograd.backward(list(outs), [up[k].to(DEV) for k in names])
        res.append({k: t.grad.detach().cpu() for k, t in leaves.items()})
    for k in ("means", "scales", "quats", "rgbs", "opacities", "uv0"):
        assert torch.equal(res[0][k], res[1][k]), f"{k}: folded AABB chain differs"
    # texel gradients combine tiles with float atomics (order-dependent rounding), unaffected by the fold
    assert grad_norm_err(res[1]["texture"], res[0]["texture"]) < 1e-6
    assert float(res[0]["means"].abs().max()) > 0


def test_geometry_outputs_off_matches(deterministic):
    """geometry_outputs=False (photometric training path): img / alpha / tex and every gradient of a
    photometric upstream are bit-identical to the full render; depth / reg / normal come back as zeros."""
    case = make_case(n=500, n_texels=25000, H=64, W=80, seed=23)
    import gstex_cuda

    v, inp = case.view, case.inp
    dv = lambda t: t.detach().to(DEV).contiguous()  # noqa: E731
    up = upstream(inp.cam.H, inp.cam.W, case.C, 4)
    res = []
    for geo in (True, False):
        t = {k: dv(getattr(inp, k)).requires_grad_(True) for k in DIFF}
        outs = gstex_cuda.texture_gaussians(
            (inp.means.shape[0], 1, case.C), dv(inp.texture_dims), t["centers"], dv(inp.extents), dv(inp.depths),
            dv(case.nth), t["rgbs"], t["opacities"], t["means"], t["scales"], inp.glob_scale, t["quats"], t["uv0"],
            dv(inp.umap), dv(inp.vmap), t["texture"], dv(v.viewmat), dv(v.c2w), v.fx, v.fy, v.cx, v.cy, inp.cam.H,
            inp.cam.W, 16, inp.settings, geometry_outputs=geo)
        img, depth, reg, alpha, tex, normal = outs
        torch.autograd.backward([img, alpha, tex], [up["img"].to(DEV), up["alpha"].to(DEV), up["tex"].to(DEV)])
        res.append((img.detach().cpu(), alpha.detach().cpu(), tex.detach().cpu(),
                    {k: t[k].grad.detach().cpu() for k in t}, depth, reg, normal))
    for a, b in zip(res[0][:3], res[1][:3]):
        assert torch.equal(a, b)
    for k in ("rgbs", "opacities", "means", "scales", "quats", "centers", "uv0"):
        assert torch.equal(res[0][3][k], res[1][3][k]), k
    assert grad_norm_err(res[1][3]["texture"], res[0][3]["texture"]) < 1e-6
    assert float(res[0][4].detach().abs().max()) > 0 and float(res[1][4].abs().max()) == 0.0
    assert float(res[1][5].abs().max()) == 0.0 and float(res[1][6].abs().max()) == 0.0
