"""Known-answer and self-consistency tests of the CPU oracle (the checker the HIP path is held to).

The reference ships no kernel tests or golden images for this path, so the
oracle is pinned here by closed-form cases, brute-force restatements and finite differences."""
import math

import numpy as np
import pytest
import torch

from gstex_amd.charts import build_charts, texture_dims_to_query
from oracle import raster as O

F64 = torch.float64


def facing_camera_case(splats, H=32, W=32, f=100.0, tex_hw=(2, 2), channels=3, settings=(1 << 9) | (1 << 10)):
    """Camera at the origin looking down +z (viewmat = [I|0]); splats = list of (xyz, s, opacity, rgb)."""
    n = len(splats)
    means = torch.tensor([s[0] for s in splats], dtype=torch.float32)
    scales = torch.tensor([[s[1], s[1], 1e-6] for s in splats], dtype=torch.float32)
    quats = torch.tensor([[1.0, 0.0, 0.0, 0.0]] * n)
    opac = torch.tensor([[s[2]] for s in splats], dtype=torch.float32)
    rgbs = torch.tensor([s[3] for s in splats], dtype=torch.float32)
    vm = torch.cat([torch.eye(3), torch.zeros(3, 1)], 1)
    cam = O.Camera(vm, f, f, W / 2, H / 2, H, W, 16, torch.zeros(3))
    centers, extents = O.aabb_2d(means, scales, 1.0, quats, cam)
    _, depths = O.project_points(means, cam)
    h, w = tex_hw
    dims = torch.tensor([[h, w, i * h * w] for i in range(n)], dtype=torch.int32)
    g = torch.Generator().manual_seed(0)
    texture = torch.rand((n * h * w, channels), generator=g)
    m = 1.0 / (2 * 3.0 * scales[:, :2])
    uv0 = torch.full((n, 1, 2), 0.5)
    umap = (m[:, 0:1] * torch.tensor([[1.0, 0.0, 0.0]]))[:, None, :]
    vmap = (m[:, 1:2] * torch.tensor([[0.0, 1.0, 0.0]]))[:, None, :]
    inp = O.RasterInputs(dims, centers.detach(), extents, depths, rgbs, opac, means, scales, 1.0, quats, uv0, umap,
                         vmap, texture, cam, settings)
    return inp


def test_single_splat_closed_form():
    z, s, o = 4.0, 0.1, 0.5
    inp = facing_camera_case([((0.0, 0.0, z), s, o, (0.2, 0.4, 0.6))])
    o32, o64, aux = O.rasterize(inp)
    px, py = 15, 15  # pixel centre (15.5, 15.5); splat centre projects to (16, 16)
    X = (px + 0.5 - 16.0) / 100.0 * z
    Y = (py + 0.5 - 16.0) / 100.0 * z
    u, v = X / s, Y / s
    rho3 = u * u + v * v
    rho2 = 2.0 * ((16.0 - 15.5) ** 2 + (16.0 - 15.5) ** 2)
    alpha = o * math.exp(-0.5 * min(rho3, rho2))
    assert rho3 < rho2
    assert o64["alpha"][py, px].item() == pytest.approx(alpha, rel=1e-6)
    np.testing.assert_allclose(o64["img"][py, px].numpy(), alpha * np.array([0.2, 0.4, 0.6]), rtol=1e-6)
    assert o64["depth"][py, px].item() == pytest.approx(alpha * z, rel=1e-6)  # hit point lies on z = 4
    np.testing.assert_allclose(o64["normal"][py, px].numpy(), [0.0, 0.0, -alpha], atol=1e-7)  # faces camera
    # texture: tu = 0.5 + (X - 0) * m, texel grid 2x2 corner-aligned, clamp to edge
    m = 1.0 / (6.0 * s)
    tu, tv = 0.5 + X * m, 0.5 + Y * m
    xx, yy = min(max(tu * 2, 0), 1), min(max(tv * 2, 0), 1)
    i0, j0 = int(xx), int(yy)
    ax, ay = xx - i0, yy - j0
    T = inp.texture.double().numpy()
    i1, j1 = min(i0 + 1, 1), min(j0 + 1, 1)
    val = (1 - ax) * ((1 - ay) * T[i0 * 2 + j0] + ay * T[i0 * 2 + j1]) + ax * ((1 - ay) * T[i1 * 2 + j0] + ay * T[i1 * 2 + j1])
    np.testing.assert_allclose(o64["tex"][py, px].numpy(), alpha * val, rtol=1e-6)
    assert o64["reg"][py, px].item() == pytest.approx(0.0, abs=1e-12)  # one contributor: no distortion
    # fp32 evaluation within 1e-6 of fp64 here
    assert (o32["img"].double() - o64["img"]).abs().max().item() < 1e-6


def test_occlusion_order_and_distortion():
    front = ((0.0, 0.0, 4.0), 0.2, 0.7, (1.0, 0.0, 0.0))
    back = ((0.0, 0.0, 6.0), 0.3, 0.6, (0.0, 1.0, 0.0))
    inp = facing_camera_case([back, front])  # input order must not matter: depth sort
    _, o64, aux = O.rasterize(inp)
    py = px = 15
    tile = (py // 16) * 2 + px // 16
    s, e = aux["tile_ranges"][tile]
    assert list(aux["sorted_ids"][s:e]) == [1, 0], "tile list must be sorted by depth"
    img = o64["img"][py, px].numpy()
    a_f = img[0]  # front is pure red
    a_b = img[1] / (1.0 - a_f)
    assert 0 < a_f < 0.7 and 0 < a_b < 0.6
    assert o64["alpha"][py, px].item() == pytest.approx(1 - (1 - a_f) * (1 - a_b), rel=1e-9)
    # distortion of two contributors = w1 w2 (m1 - m2)^2 with m = far/(far-near) (1 - near/z)
    zf = o64["depth"][py, px].item()
    mf = float(O.K_FAR_RATIO) * (1 - 0.2 / 4.0)
    mb = float(O.K_FAR_RATIO) * (1 - 0.2 / 6.0)
    w_f, w_b = a_f, (1 - a_f) * a_b
    assert zf == pytest.approx(w_f * 4.0 + w_b * 6.0, rel=1e-6)
    assert o64["reg"][py, px].item() == pytest.approx(w_f * w_b * (mf - mb) ** 2, rel=1e-5)


def test_early_termination_at_t_min():
    stack = [((0.0, 0.0, 4.0 + 0.5 * i), 0.5, 0.98, (1.0, 1.0, 1.0)) for i in range(6)]
    inp = facing_camera_case(stack)
    o32, o64, aux = O.rasterize(inp)
    py = px = 15
    # alpha ~ 0.978 per splat: T = 2.2e-2, 4.7e-4, then 1.0e-5 < 1e-4 -> the third splat stops the pixel
    assert int(aux["last"][py, px]) == 1
    a = float(o64["img"][py, px, 0])  # = 1 - T after two splats (white, no background)
    assert o64["alpha"][py, px].item() == pytest.approx(a, rel=1e-9)
    assert 1 - a > 1e-4


def test_alpha_clamp_and_fp32_threshold():
    # opacity 1 clamps alpha to 0.99: in fp32 (1 - 0.99f)^2 = 9.99998e-5 < 1e-4, so ONE splat
    # already terminates the pixel (the second never contributes)
    stack = [((0.0, 0.0, 4.0 + 0.5 * i), 0.5, 1.0, (1.0, 1.0, 1.0)) for i in range(3)]
    inp = facing_camera_case(stack)
    o32, _, aux = O.rasterize(inp)
    assert int(aux["last"][15, 15]) == 0
    assert o32["alpha"][15, 15].item() == pytest.approx(float(np.float32(0.99)), rel=1e-7)


def brute_bins(centers, extents, depths, H, W):
    tx_n, ty_n = (W + 15) // 16, (H + 15) // 16
    c = centers.numpy().astype(np.float32)
    e = extents.numpy().astype(np.float32)
    pairs = []
    for g in range(c.shape[0]):
        if not (e[g, 0] > 0 and e[g, 1] > 0):
            continue
        x0 = int(min(max(c[g, 0] / np.float32(16) - e[g, 0] / np.float32(16), 0), tx_n))
        x1 = int(min(max(c[g, 0] / np.float32(16) + e[g, 0] / np.float32(16) + np.float32(1), 0), tx_n))
        y0 = int(min(max(c[g, 1] / np.float32(16) - e[g, 1] / np.float32(16), 0), ty_n))
        y1 = int(min(max(c[g, 1] / np.float32(16) + e[g, 1] / np.float32(16) + np.float32(1), 0), ty_n))
        for ty in range(y0, y1):
            for tx in range(x0, x1):
                pairs.append((ty * tx_n + tx, np.float32(depths[g]).view(np.uint32), g))
    pairs.sort()
    return pairs, tx_n * ty_n


def test_binning_matches_brute_force():
    from gstex_amd.scene import make_scene, sphere_view

    sc = make_scene(300, 0, seed=3)
    v = sphere_view(2, 48, 64)
    means, scales, quats, _ = sc.activated()
    cam = O.Camera(v.viewmat, v.fx, v.fy, v.cx, v.cy, 48, 64, 16, v.c2w[:3, 3])
    c, e = O.aabb_2d(means, scales, 1.0, quats, cam)
    _, d = O.project_points(means, cam)
    off, tr, ids, slots = O.bin_and_sort(c, e, d, 48, 64)
    pairs, n_tiles = brute_bins(c.detach(), e, d, 48, 64)
    assert len(pairs) == len(ids) == int(O.num_tiles_hit(c, e, 48, 64).sum())
    assert [p[2] for p in pairs] == list(ids)
    counts = np.bincount([p[0] for p in pairs], minlength=n_tiles)
    assert np.array_equal(tr[:, 1] - tr[:, 0], counts)
    # slots are a permutation of the gid-major emission order
    assert sorted(slots.tolist()) == list(range(len(ids)))


def test_gradients_match_finite_differences():
    from helpers import make_case

    case = make_case(n=12, n_texels=600, H=24, W=24, seed=21, opacity=None)
    inp = case.inp
    bins = O.bin_and_sort(inp.centers, inp.extents, inp.depths, 24, 24)
    dec = O._render(inp, torch.float32, bins[1], bins[2], None)["decisions"]
    g = torch.Generator().manual_seed(1)
    up = {k: torch.randn(s, generator=g, dtype=F64) for k, s in
          [("img", (24, 24, 3)), ("depth", (24, 24)), ("reg", (24, 24)), ("alpha", (24, 24)), ("tex", (24, 24, 3)),
           ("normal", (24, 24, 3))]}
    names = ["means", "scales", "quats", "opacities", "rgbs", "texture", "centers"]
    base = {k: getattr(inp, k).double() for k in names}

    def loss(vals):
        for k in names:
            setattr(inp, k, vals[k])
        out = O._render(inp, F64, bins[1], bins[2], dec)["out"]
        return sum((out[k] * up[k]).sum() for k in up)

    leaves = {k: v.clone().requires_grad_(True) for k, v in base.items()}
    loss(leaves).backward()
    rng = np.random.default_rng(0)
    eps = 1e-6
    for k in names:
        flat = base[k].reshape(-1)
        for idx in rng.choice(flat.numel(), size=min(4, flat.numel()), replace=False):
            def shifted(delta):
                vals = {kk: vv.clone() for kk, vv in base.items()}
                vals[k].reshape(-1)[idx] += delta
                return loss(vals).item()
            fd = (shifted(eps) - shifted(-eps)) / (2 * eps)
            ad = leaves[k].grad.reshape(-1)[idx].item()
            assert abs(fd - ad) <= 1e-5 * max(1.0, abs(ad)), f"{k}[{idx}]: autograd {ad} vs fd {fd}"


def test_settings_bits_semantics():
    from helpers import make_case

    noaa = make_case(n=80, n_texels=2000, H=32, W=32, seed=4, settings=1 << 10)
    _, o, _ = O.rasterize(noaa.inp)
    noreg = make_case(n=80, n_texels=2000, H=32, W=32, seed=4, settings=1 << 9)
    _, o2, _ = O.rasterize(noreg.inp)
    assert torch.all(o2["reg"] == 0)
    assert o["reg"].abs().sum() > 0
    # without the low-pass the splat centre (centers input) does not influence the image
    c = noaa.inp.centers.clone().double().requires_grad_(True)
    noaa.inp.centers = c
    _, o3, _ = O.rasterize(noaa.inp)
    o3["img"].sum().backward()
    assert c.grad is None or torch.all(c.grad == 0)


def test_texture_sample_identity_on_same_charts():
    log_scales = torch.log(10 ** (-2.5 + 1.5 * torch.rand((50, 3), generator=torch.Generator().manual_seed(2))))
    dims, _, _ = build_charts(log_scales, 3000)
    T = int((dims[:, 0] * dims[:, 1]).sum())
    tex = torch.rand(T, 3, generator=torch.Generator().manual_seed(3))
    ids, uv = texture_dims_to_query(dims)
    out = O.texture_sample(dims[ids], tex, uv)
    # texel centres come back up to the fp32 rounding of uv * h - 0.5 (|err| <= h * 2^-24 per coordinate, h <= 256
    # here): a bilinear weight of that size on the neighbour
    assert torch.allclose(out, tex, atol=2e-5), "resampling onto identical charts must be the identity"


def test_sh_low_orders():
    dirs = torch.tensor([[0.0, 0.0, 2.0], [3.0, 0.0, 0.0], [0.0, -1.0, 0.0]])
    coeffs = torch.zeros(3, 16, 3)
    coeffs[:, 0] = 1.0
    coeffs[:, 2] = 1.0  # the z basis
    out0 = O.spherical_harmonics(0, dirs, coeffs)
    assert torch.allclose(out0, torch.full((3, 3), float(O.SH_C0)))
    out1 = O.spherical_harmonics(1, dirs, coeffs)
    expect_z = torch.tensor([1.0, 0.0, 0.0])[:, None] * float(O.SH_C1)
    assert torch.allclose(out1, float(O.SH_C0) + expect_z, atol=1e-6)


def test_texture_edit_uniform_stroke_known_answer():
    # one opaque-ish splat facing the camera, 4x4 texels; a uniform stroke (a = 1, rgb = c) over the
    # whole image with an open depth window: every touched texel gets colour c and blend weight 1
    inp = facing_camera_case([((0.0, 0.0, 2.0), 0.05, 0.8, (0.1, 0.2, 0.3))], tex_hw=(4, 4), settings=1 << 13)
    H, W = inp.cam.H, inp.cam.W
    c = torch.tensor([0.2, 0.4, 0.6])
    rgb = c.expand(H, W, 3).clone()
    a = torch.ones(H, W)
    out = O.texture_edit(inp, rgb, a, torch.full((H, W), -1e9), torch.full((H, W), 1e9))
    touched = out[:, 4] > 0
    assert int(touched.sum()) == 16, "every texel of the block is reached"
    assert torch.allclose(out[touched, 3] / out[touched, 4], torch.ones(16, dtype=F64), atol=1e-6)
    col = out[touched, :3] / out[touched, 3:4]
    assert torch.allclose(col, c.to(F64).expand_as(col), atol=1e-6)
    # half-transparent stroke: weight a; closed depth window: nothing
    out2 = O.texture_edit(inp, rgb, torch.full((H, W), 0.25), torch.full((H, W), -1e9), torch.full((H, W), 1e9))
    assert torch.allclose(out2[touched, 3] / out2[touched, 4], torch.full((16,), 0.25, dtype=F64), atol=1e-6)
    out3 = O.texture_edit(inp, rgb, a, torch.full((H, W), 2.5), torch.full((H, W), 3.0))
    assert float(out3.abs().sum()) == 0.0
    # total weight: sum_texels out[:, 4] = sum_pixels w (bilinear weights sum to 1 per pair)
    fwd = O._render(inp, torch.float32, *O.bin_and_sort(inp.centers, inp.extents, inp.depths, H, W)[1:3], None)
    assert abs(float(out[:, 4].sum()) - float(fwd["out"]["alpha"].double().sum())) < 1e-4


def test_near_edge_on_rows_change_only_the_ill_conditioned_pairs():
    """RasterInputs.hp (raster.hip hit_p_hp: near-edge-on splats' p from their fp64 row, rounded once): the fp32 pass
    moves by fp32 noise only (the fp64 evaluation is the same function), and only pixels of marked splats move."""
    import sys
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from helpers import make_case

    case = make_case(n=300, n_texels=20000, H=48, W=48, seed=12)
    tab = O._splat_table(case.inp, F64)
    assert 0 < int(tab["hp"].sum()) < case.inp.means.shape[0], "the scene must hold marked and unmarked splats"
    with_hp, _, aux = O.rasterize(case.inp)
    case.inp.hp = False
    without, _, _ = O.rasterize(case.inp)
    ok = aux["margin"] >= 1e-5
    moved = False
    for k in ("img", "alpha", "depth", "tex", "normal"):
        d = (with_hp[k].double() - without[k].double()).abs()
        d = d[ok] if d.dim() == 2 else d[ok]
        assert float(d.max()) <= 1e-5, k
        moved |= bool((d > 0).any())
    assert moved, "some near-edge-on pair must change in its last bits"
