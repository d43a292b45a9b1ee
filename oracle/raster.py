"""CPU restatement of the textured-2DGS rasterizer (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Follows, op for op in fp32, the device functions of gstex_amd/csrc/gstex_common.h, raster.hip,
preprocess.hip and binning.hip, which in turn implement the call-site contracts of
nerfstudio/models/gstex.py:1059-1170.

Parity unpinned w.r.t. the reference CUDA rasterizer (absent from /root/reference).

Forward values are computed in fp32 with the same operation order as the kernels (correctly rounded
division and sqrt), so the threshold decisions (alpha >= 1/255, T < 1e-4, z >= near, AA branch, texel
cell) match the GPU except within a few ulps of a threshold: the kernels evaluate exp and the pair's
1 / p.z with the hardware v_exp_f32 / v_rcp_f32, a few ulps from this restatement; each pixel's smallest
decision margin is reported (aux["margin"]) so tests can tell such a flip from a defect.
Gradients come from torch autograd of an fp64 re-evaluation that reuses those fp32 decisions —
i.e. the exact-arithmetic gradient of the function the GPU evaluates.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

F32 = torch.float32
F64 = torch.float64

# constants of gstex_common.h, rounded to fp32 exactly like the C++ constexprs
K_TILE = 16
K_CUTOFF2 = np.float32(9.0)
K_MIN_EXTENT = np.float32(2.1213180)
K_NEAR = np.float32(0.2)
K_FAR_RATIO = np.float32(np.float32(100.0) / np.float32(99.8))
K_ALPHA_MAX = np.float32(0.99)
K_ALPHA_MIN = np.float32(np.float32(1.0) / np.float32(255.0))
K_TMIN = np.float32(1e-4)
K_FILTER_INV_SQ = np.float32(2.0)
K_PROJ_CLIP = np.float32(0.01)

SETTING_AA_BLUR = 1 << 9
SETTING_DIST_REG = 1 << 10
SETTING_EVAL_NORMAL = 1 << 15  # gstex.py:1198 eval render: unit-length normal output


def _c(v, dtype):
    return torch.tensor(float(v), dtype=dtype)


def _arg32(v, dtype):
    """A scalar kernel argument (fx, fy, cx, cy, glob_scale): the reference's extension takes them as C `float`
    (gsplat-0.1's bindings, which gstex_cuda extends: `const float fx, ... const float glob_scale`; gstex.py:1142-1160
    passes Python floats), so every precision evaluates with the fp32-rounded value -- also include/gstex_hip.h's
    gstex_camera and glob_scale arguments."""
    return torch.tensor(float(np.float32(v)), dtype=dtype)


def _div(a, b):
    """fp32 a / b correctly rounded on any host (torch's vectorised fp32 division/sqrt are not
    correctly rounded on every CPU; the GPU's are).  Exact: fp64 has > 2*24+2 bits."""
    if isinstance(a, torch.Tensor) and a.dtype == F32 or isinstance(b, torch.Tensor) and b.dtype == F32:
        ad = a.double() if isinstance(a, torch.Tensor) else float(a)
        bd = b.double() if isinstance(b, torch.Tensor) else float(b)
        return (ad / bd).float()
    return a / b


def _fma(a, b, c):
    """fp32 fused multiply-add (a * b + c, one rounding) as raster.hip's __builtin_fmaf: the fp64 product is exact
    and the fp64 sum's own rounding can change the fp32 result only at a rounding midpoint (p < 2^-28)."""
    if isinstance(a, torch.Tensor) and a.dtype == F32:
        return (a.double() * b.double() + (c.double() if isinstance(c, torch.Tensor) else float(c))).float()
    return a * b + c


def _sqrt(a):
    if a.dtype == F32:
        return torch.sqrt(a.double()).float()
    return torch.sqrt(a)


# ----------------------------------------------------------------------------------------
# per-splat geometry (gstex_common.h: quat_frame, splat_homography, aabb_from_homog, tile_rect)
# ----------------------------------------------------------------------------------------
def quat_frame(q: torch.Tensor):
    """wxyz quaternion (N,4) -> rotation columns t_u, t_v, t_w (N,3).  gstex_common.h:quat_frame;
    equals nerfstudio/utils/rotations.py:43-72 on unit quaternions."""
    w, x, y, z = q.unbind(-1)
    nrm = _sqrt(((w * w + x * x) + y * y) + z * z)
    w, x, y, z = _div(w, nrm), _div(x, nrm), _div(y, nrm), _div(z, nrm)
    r00 = 1.0 - 2.0 * (y * y + z * z)
    r01 = 2.0 * (x * y - w * z)
    r02 = 2.0 * (x * z + w * y)
    r10 = 2.0 * (x * y + w * z)
    r11 = 1.0 - 2.0 * (x * x + z * z)
    r12 = 2.0 * (y * z - w * x)
    r20 = 2.0 * (x * z - w * y)
    r21 = 2.0 * (y * z + w * x)
    r22 = 1.0 - 2.0 * (x * x + y * y)
    tu = torch.stack([r00, r10, r20], -1)
    tv = torch.stack([r01, r11, r21], -1)
    tw = torch.stack([r02, r12, r22], -1)
    return tu, tv, tw


def _vrow(V, r, a):
    return (V[r, 0] * a[..., 0] + V[r, 1] * a[..., 1]) + V[r, 2] * a[..., 2]


def _dot3(a, b):
    return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


@dataclass
class Camera:
    viewmat: torch.Tensor  # (3,4)
    fx: float
    fy: float
    cx: float
    cy: float
    H: int
    W: int
    block: int = K_TILE
    campos: torch.Tensor | None = None  # (3,) = c2w[:3,3]

    def cast(self, dtype):
        V = self.viewmat.to(dtype)
        cp = self.campos.to(dtype) if self.campos is not None else -(V[:, :3].T @ V[:, 3])
        return V, cp, _arg32(self.fx, dtype), _arg32(self.fy, dtype), _arg32(self.cx, dtype), _arg32(self.cy, dtype)


def splat_homography(means, scales, glob_scale, quats, cam: Camera, dtype=F32):
    """M = K [R|t] [[su t_u, sv t_v, mu],[0,0,1]] -> rows (Tu, Tv, Tw), each (N,3).
    gstex_common.h:splat_homography."""
    V, _, fx, fy, cx, cy = cam.cast(dtype)
    tu, tv, _ = quat_frame(quats.to(dtype))
    glob = _arg32(glob_scale, dtype)
    su = scales[:, 0].to(dtype) * glob
    sv = scales[:, 1].to(dtype) * glob
    a = tu * su[:, None]
    b = tv * sv[:, None]
    mu = means.to(dtype)
    W0 = [_vrow(V, r, a) for r in range(3)]
    W1 = [_vrow(V, r, b) for r in range(3)]
    W2 = [_vrow(V, r, mu) + V[r, 3] for r in range(3)]
    Tu = torch.stack([fx * W0[0] + cx * W0[2], fx * W1[0] + cx * W1[2], fx * W2[0] + cx * W2[2]], -1)
    Tv = torch.stack([fy * W0[1] + cy * W0[2], fy * W1[1] + cy * W1[2], fy * W2[1] + cy * W2[2]], -1)
    Tw = torch.stack([W0[2], W1[2], W2[2]], -1)
    return Tu, Tv, Tw


def splat_anchored(means, scales, glob_scale, quats, cam: Camera, dtype=F32):
    """Anchored homography (gstex_common.h:splat_anchored): Tu' = Tu - xa Tw, Tv' = Tv - ya Tw with
    the anchor (xa, ya) = projection of the splat centre; returns (Tu', Tv', Tw, xa, ya)."""
    V, _, fx, fy, cx, cy = cam.cast(dtype)
    tu, tv, _ = quat_frame(quats.to(dtype))
    glob = _arg32(glob_scale, dtype)
    su = scales[:, 0].to(dtype) * glob
    sv = scales[:, 1].to(dtype) * glob
    a = tu * su[:, None]
    b = tv * sv[:, None]
    mu = means.to(dtype)
    W0 = [_vrow(V, r, a) for r in range(3)]
    W1 = [_vrow(V, r, b) for r in range(3)]
    W2 = [_vrow(V, r, mu) + V[r, 3] for r in range(3)]
    xn = _div(W2[0], W2[2])
    yn = _div(W2[1], W2[2])
    zero = torch.zeros_like(xn)
    Tu = torch.stack([fx * (W0[0] - xn * W0[2]), fx * (W1[0] - xn * W1[2]), zero], -1)
    Tv = torch.stack([fy * (W0[1] - yn * W0[2]), fy * (W1[1] - yn * W1[2]), zero], -1)
    Tw = torch.stack([W0[2], W1[2], W2[2]], -1)
    return Tu, Tv, Tw, fx * xn + cx, fy * yn + cy


def project_points(means, cam: Camera, dtype=F32):
    """gstex_cuda.get_aabb_2d.project_points (gstex.py:1077) -> xys (N,2), depths (N,)."""
    V, _, fx, fy, cx, cy = cam.cast(dtype)
    mu = means.to(dtype)
    x = _vrow(V, 0, mu) + V[0, 3]
    y = _vrow(V, 1, mu) + V[1, 3]
    z = _vrow(V, 2, mu) + V[2, 3]
    ok = z > _c(K_PROJ_CLIP, dtype)
    zs = torch.where(ok, z, torch.ones_like(z))
    xs = torch.where(ok, fx * _div(x, zs) + cx, torch.zeros_like(x))
    ys = torch.where(ok, fy * _div(y, zs) + cy, torch.zeros_like(y))
    return torch.stack([xs, ys], -1), z


def aabb_2d(means, scales, glob_scale, quats, cam: Camera, dtype=F32):
    """gstex_cuda.get_aabb_2d.get_aabb_2d (gstex.py:1079): 2DGS compute_aabb at the 3-sigma
    cutoff.  Culled splats (centre at/behind near, or disc crossing the camera plane) get
    centre = extent = 0.  Differentiable w.r.t. means/scales/quats through the centre."""
    Tu, Tv, Tw = splat_homography(means, scales, glob_scale, quats, cam, dtype)
    c9 = _c(K_CUTOFF2, dtype)
    d = (c9 * (Tw[:, 0] * Tw[:, 0]) + c9 * (Tw[:, 1] * Tw[:, 1])) - Tw[:, 2] * Tw[:, 2]
    ok = (Tw[:, 2] > _c(K_NEAR, dtype)) & (d < 0)
    ds = torch.where(ok, d, -torch.ones_like(d))
    fxy = _div(c9, ds)
    fz = _div(_c(-1.0, dtype), ds)
    px = (fxy * (Tu[:, 0] * Tw[:, 0]) + fxy * (Tu[:, 1] * Tw[:, 1])) + fz * (Tu[:, 2] * Tw[:, 2])
    py = (fxy * (Tv[:, 0] * Tw[:, 0]) + fxy * (Tv[:, 1] * Tw[:, 1])) + fz * (Tv[:, 2] * Tw[:, 2])
    qx = (fxy * (Tu[:, 0] * Tu[:, 0]) + fxy * (Tu[:, 1] * Tu[:, 1])) + fz * (Tu[:, 2] * Tu[:, 2])
    qy = (fxy * (Tv[:, 0] * Tv[:, 0]) + fxy * (Tv[:, 1] * Tv[:, 1])) + fz * (Tv[:, 2] * Tv[:, 2])
    ex = _sqrt(torch.clamp(px * px - qx, min=1e-4))
    ey = _sqrt(torch.clamp(py * py - qy, min=1e-4))
    me = _c(K_MIN_EXTENT, dtype)
    ex = torch.maximum(ex, me)
    ey = torch.maximum(ey, me)
    z = torch.zeros_like(px)
    centers = torch.stack([torch.where(ok, px, z), torch.where(ok, py, z)], -1)
    extents = torch.stack([torch.where(ok, ex, z), torch.where(ok, ey, z)], -1).detach()
    return centers, extents


def tile_rects(centers: np.ndarray, extents: np.ndarray, H: int, W: int, block: int):
    """gstex_common.h:tile_rect (gsplat-0.1 get_tile_bbox convention), numpy fp32."""
    tiles_x = (W + block - 1) // block
    tiles_y = (H + block - 1) // block
    c = np.asarray(centers, dtype=np.float32)
    e = np.asarray(extents, dtype=np.float32)
    b = np.float32(block)
    tc = c / b
    tr = e / b
    one = np.float32(1.0)

    def cl(v, hi):
        return np.minimum(np.maximum(v, np.float32(0.0)), np.float32(hi)).astype(np.int64)

    with np.errstate(invalid="ignore"):
        x0 = cl(np.nan_to_num(tc[:, 0] - tr[:, 0], nan=0.0), tiles_x)
        x1 = cl(np.nan_to_num(tc[:, 0] + tr[:, 0] + one, nan=0.0), tiles_x)
        y0 = cl(np.nan_to_num(tc[:, 1] - tr[:, 1], nan=0.0), tiles_y)
        y1 = cl(np.nan_to_num(tc[:, 1] + tr[:, 1] + one, nan=0.0), tiles_y)
    valid = (e[:, 0] > 0) & (e[:, 1] > 0)
    x1 = np.maximum(x1, x0)
    y1 = np.maximum(y1, y0)
    x0 = np.where(valid, x0, 0); x1 = np.where(valid, x1, 0)
    y0 = np.where(valid, y0, 0); y1 = np.where(valid, y1, 0)
    return x0, x1, y0, y1, tiles_x, tiles_y


def num_tiles_hit(centers, extents, H, W, block=K_TILE):
    """gstex_cuda.get_aabb_2d.get_num_tiles_hit_2d (gstex.py:1080) -> int32 (N,)."""
    x0, x1, y0, y1, _, _ = tile_rects(_np(centers), _np(extents), H, W, block)
    return torch.from_numpy(((x1 - x0) * (y1 - y0)).astype(np.int32))


def _np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


def bin_and_sort(centers, extents, depths, H, W, block=K_TILE):
    """Tile binning + per-tile depth sort (inside texture_gaussians; gstex.py:1136-1139,1158).
    Returns (offsets (N+1,), tile_ranges (n_tiles,2), sorted_ids (I,), sorted_slots (I,)) as int32
    numpy arrays.  Order per tile: ascending (float bits of depth, splat id) — a stable sort of
    the gid-major emission by (tile << 32 | depth_bits), as in the gsplat-0.1 lineage."""
    x0, x1, y0, y1, tiles_x, tiles_y = tile_rects(_np(centers), _np(extents), H, W, block)
    nx = x1 - x0
    cnt = nx * (y1 - y0)
    n = cnt.shape[0]
    offsets = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(cnt, out=offsets[1:])
    total = int(offsets[-1])
    n_tiles = tiles_x * tiles_y
    if total == 0:
        return (offsets.astype(np.int32), np.zeros((n_tiles, 2), np.int32), np.zeros(0, np.int32),
                np.zeros(0, np.int32))
    gid = np.repeat(np.arange(n, dtype=np.int64), cnt)
    local = np.arange(total, dtype=np.int64) - offsets[:-1][gid]
    nxg = np.maximum(nx[gid], 1)
    ty = y0[gid] + local // nxg
    tx = x0[gid] + local % nxg
    tile = ty * tiles_x + tx
    dbits = np.asarray(_np(depths), dtype=np.float32).view(np.uint32).astype(np.uint64)
    order = np.lexsort((gid, dbits[gid], tile))
    sorted_ids = gid[order].astype(np.int32)
    sorted_slots = np.arange(total, dtype=np.int64)[order].astype(np.int32)
    tcount = np.bincount(tile, minlength=n_tiles)
    starts = np.zeros(n_tiles + 1, dtype=np.int64)
    np.cumsum(tcount, out=starts[1:])
    tile_ranges = np.stack([starts[:-1], starts[1:]], -1).astype(np.int32)
    return offsets.astype(np.int32), tile_ranges, sorted_ids, sorted_slots


# ----------------------------------------------------------------------------------------
# rasterizer
# ----------------------------------------------------------------------------------------
@dataclass
class RasterInputs:
    texture_dims: torch.Tensor  # (N,3) int32 [h, w, off]
    centers: torch.Tensor       # (N,2)
    extents: torch.Tensor       # (N,2)
    depths: torch.Tensor        # (N,)
    rgbs: torch.Tensor          # (N,3)
    opacities: torch.Tensor     # (N,1)
    means: torch.Tensor         # (N,3)
    scales: torch.Tensor        # (N,3)
    glob_scale: float
    quats: torch.Tensor         # (N,4)
    uv0: torch.Tensor           # (N,1,2)
    umap: torch.Tensor          # (N,1,3)
    vmap: torch.Tensor          # (N,1,3)
    texture: torch.Tensor       # (T,C)
    cam: Camera
    settings: int = SETTING_AA_BLUR | SETTING_DIST_REG
    background: torch.Tensor | None = None  # (3,)
    # near-edge-on splats (|normal . view direction| < K_HP_COS) evaluated with their homogeneous point p from the
    # fp64 record (raster.hip hit_p_hp, gstex_raster_setup's hp_records): what texture_gaussians does; texture_edit
    # (records without hp rows) does not
    hp: bool = True


# raster.hip setup_kernel evaluates the per-splat record in fp64 and rounds each value to fp32 once (and
# setup_bwd_chain differentiates it in fp64): the fp32 evaluation of the record was measured to dominate the
# means / quats gradient error (tools/grad_precision.py).  False restores the all-fp32 record
# (precision analysis only).
RECORD_FP64 = True
# gstex_common.h kHpCos: splats with |normal . unit view direction| below it are near edge-on
K_HP_COS = 0.1
# Precision analysis only (tools/grad_precision.py --hp-sum32): the gradient of a near-edge-on splat's fp64 homogeneous
# point p w.r.t. its fp64 record (A, B, Pz) formed as the HIP backward forms it -- fp32 products dp * dx summed over a
# tile's pixels in fp32, the anchor held constant -- instead of autograd's fp64 products and sums.
HP_SUM32 = False
# Precision analysis only (tools/hp_sum_model.py): a list that the fp32 gradient pass appends, per tile, the pairs'
# splat ids, pixel offsets from the anchor (fp32 and fp64) and -- through hooks -- dL/dp.  None = off.
CAPTURE = None


class _HpPoint(torch.autograd.Function):
    """p = dx A + dy B + (0, 0, Pz) in fp64, rounded to fp32; backward in fp32 per tile (HP_SUM32)."""

    @staticmethod
    def forward(ctx, dx64, dy64, A64, B64, Pz64):
        ctx.save_for_backward(dx64.float(), dy64.float())
        p = torch.stack([dx64 * A64[..., 0] + dy64 * B64[..., 0], dx64 * A64[..., 1] + dy64 * B64[..., 1],
                         dy64 * B64[..., 2] + (dx64 * A64[..., 2] + Pz64)], -1)
        return p.float()

    @staticmethod
    def backward(ctx, gp):
        dx, dy = ctx.saved_tensors
        gA = (gp * dx[..., None]).sum(1, keepdim=True)
        gB = (gp * dy[..., None]).sum(1, keepdim=True)
        gP = gp[..., 2].sum(1, keepdim=True)
        return None, None, gA.double(), gB.double(), gP.double()


def _splat_table(inp: RasterInputs, dtype):
    """gstex_amd/csrc/raster.hip:setup_kernel — per-splat record in `dtype` (fp32: fp64 evaluation, rounded once)."""
    if dtype == F32 and RECORD_FP64:
        return {k: (v.to(F32) if v.is_floating_point() else v) for k, v in _splat_table(inp, F64).items()}
    V, campos, fx, fy, cx, cy = inp.cam.cast(dtype)
    Tu, Tv, Tw, xa, ya = splat_anchored(inp.means, inp.scales, inp.glob_scale, inp.quats, inp.cam, dtype)
    tu, tv, tw = quat_frame(inp.quats.to(dtype))
    glob = _arg32(inp.glob_scale, dtype)
    su = inp.scales[:, 0].to(dtype) * glob
    sv = inp.scales[:, 1].to(dtype) * glob
    mu = inp.means.to(dtype)
    dirv = campos[None, :] - mu
    sgn = torch.where(_dot3(tw, dirv) < 0, -1.0, 1.0).to(dtype).detach()
    # splat_math.h splat_record: |tw . dir| < kHpCos |dir| (fp64)
    with torch.no_grad():
        hp = _dot3(tw, dirv).abs() < K_HP_COS * torch.sqrt(_dot3(dirv, dirv))
    um = inp.umap[:, 0, :].to(dtype).detach()
    vm = inp.vmap[:, 0, :].to(dtype).detach()
    # the texture affine prescaled to texel units (raster.hip setup_kernel): the sample point (tu h, tv w)
    hd = inp.texture_dims[:, 0].to(dtype)
    wd = inp.texture_dims[:, 1].to(dtype)
    # affine form of the homography (gstex_common.h affine_homog): p = dx A + dy B + (0, 0, Pz)
    A = torch.stack([Tw[:, 2] * Tv[:, 1], -(Tw[:, 2] * Tv[:, 0]), Tw[:, 1] * Tv[:, 0] - Tw[:, 0] * Tv[:, 1]], -1)
    B = torch.stack([-(Tu[:, 1] * Tw[:, 2]), Tu[:, 0] * Tw[:, 2], Tu[:, 1] * Tw[:, 0] - Tu[:, 0] * Tw[:, 1]], -1)
    Pz = Tu[:, 0] * Tv[:, 1] - Tu[:, 1] * Tv[:, 0]
    return dict(
        A=A, B=B, Pz=Pz, Tw=Tw, xa=xa, ya=ya,
        xy=inp.centers.to(dtype),
        opac=inp.opacities[:, 0].to(dtype),
        rgb=inp.rgbs.to(dtype),
        nrm=tw * sgn[:, None],
        tu0=inp.uv0[:, 0, 0].to(dtype) * hd, tv0=inp.uv0[:, 0, 1].to(dtype) * wd,
        auu=su * _dot3(tu, um) * hd, auv=sv * _dot3(tv, um) * hd,
        avu=su * _dot3(tu, vm) * wd, avv=sv * _dot3(tv, vm) * wd,
        sgn=sgn, hp=hp,
    )


def rasterize(inp: RasterInputs, grad_dtype=F64, bins=None, table_dtype=None):
    """Forward composite.  Returns (outputs_fp32, outputs_hi, aux) where outputs_* is a dict
    img (H,W,3), depth, reg, alpha (H,W), tex (H,W,C), normal (H,W,3); outputs_fp32 are the values
    the GPU must reproduce, outputs_hi the `grad_dtype` re-evaluation (differentiable w.r.t. the
    leaf tensors of `inp` that require grad) that shares the fp32 decisions.
    table_dtype (precision analysis, tools/grad_precision.py): evaluate the per-splat table (the chain that
    raster.hip's setup / setup_bwd implement) in this dtype and only the per-pair part in grad_dtype."""
    cam = inp.cam
    H, W = cam.H, cam.W
    if bins is None:
        bins = bin_and_sort(inp.centers, inp.extents, inp.depths, H, W, cam.block)
    offsets, tile_ranges, sorted_ids, sorted_slots = bins
    dec = _render(inp, F32, tile_ranges, sorted_ids, None)
    hi = _render(inp, grad_dtype, tile_ranges, sorted_ids, dec["decisions"], table_dtype=table_dtype)
    aux = dict(offsets=offsets, tile_ranges=tile_ranges, sorted_ids=sorted_ids, sorted_slots=sorted_slots,
               last=dec["last"], T_final=dec["out"]["T_final"], margin=dec["margin"])
    return dec["out"], hi["out"], aux


def _render(inp: RasterInputs, dtype, tile_ranges, sorted_ids, decisions, edit=None, table_dtype=None):
    cam = inp.cam
    H, W = cam.H, cam.W
    C = inp.texture.shape[1]
    aa = bool(inp.settings & SETTING_AA_BLUR)
    dreg = bool(inp.settings & SETTING_DIST_REG)
    tab64 = None
    if inp.hp and dtype == F32 and RECORD_FP64 and table_dtype in (None, F32):
        # the fp32 record is the fp64 one rounded (setup_kernel); near-edge-on splats' p comes from the fp64 one
        tab64 = _splat_table(inp, F64)
        tab = {k: (v.to(F32) if v.is_floating_point() else v) for k, v in tab64.items()}
    elif table_dtype is None or table_dtype == dtype:
        tab = _splat_table(inp, dtype)
    else:  # mixed precision: table in table_dtype, cast (differentiably) to the per-pair dtype
        tab = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in _splat_table(inp, table_dtype).items()}
    if decisions is not None:  # orientation sign from the fp32 pass
        tab["nrm"] = (tab["nrm"] * tab["sgn"][:, None]) * decisions["sgn"][:, None]
    tex = inp.texture.to(dtype)
    tdims = inp.texture_dims.long()
    bg = inp.background.to(dtype) if inp.background is not None else torch.zeros(3, dtype=dtype)
    tiles_x = (W + K_TILE - 1) // K_TILE
    n_tiles = tile_ranges.shape[0]

    c = lambda v: _c(v, dtype)  # noqa: E731
    near, amin, amax, tmin = c(K_NEAR), c(K_ALPHA_MIN), c(K_ALPHA_MAX), c(K_TMIN)
    fis, far = c(K_FILTER_INV_SQ), c(K_FAR_RATIO)

    pix_idx, rows = [], {k: [] for k in ["img", "depth", "reg", "T", "tex", "normal", "M1", "M2"]}
    last_all, margin_all = [], []
    new_dec = {"tiles": {}, "sgn": tab["sgn"].detach().to(F32)} if decisions is None else None
    for t in range(n_tiles):
        s, e = int(tile_ranges[t, 0]), int(tile_ranges[t, 1])
        tx, ty = t % tiles_x, t // tiles_x
        ly, lx = np.meshgrid(np.arange(K_TILE), np.arange(K_TILE), indexing="ij")
        pxi = (tx * K_TILE + lx).reshape(-1)
        pyi = (ty * K_TILE + ly).reshape(-1)
        inside = (pxi < W) & (pyi < H)
        pxi, pyi = pxi[inside], pyi[inside]
        if pxi.size == 0:
            continue
        P = pxi.size
        pix_idx.append(torch.from_numpy(pyi * W + pxi))
        if e == s:
            z = torch.zeros(P, dtype=dtype)
            rows["img"].append(torch.zeros(P, 3, dtype=dtype) + bg[None, :])
            rows["depth"].append(z); rows["reg"].append(z); rows["T"].append(torch.ones(P, dtype=dtype))
            rows["tex"].append(torch.zeros(P, C, dtype=dtype)); rows["normal"].append(torch.zeros(P, 3, dtype=dtype))
            rows["M1"].append(z); rows["M2"].append(z)
            last_all.append(torch.full((P,), -1, dtype=torch.int64))
            margin_all.append(torch.full((P,), float("inf")))
            continue
        ids = torch.from_numpy(np.asarray(sorted_ids[s:e], dtype=np.int64))
        K = ids.numel()
        # pixel (x, y) is evaluated at its centre (x + 0.5, y + 0.5): the convention of the reference's own
        # depths_to_points (gstex.py:138-139, ray through (j - cx + 0.5) / fx), DESIGN.md §1 lineage table
        px = (torch.from_numpy(pxi.astype(np.float32)) + 0.5).to(dtype)[None, :]  # exact in fp32
        py = (torch.from_numpy(pyi.astype(np.float32)) + 0.5).to(dtype)[None, :]
        g = {k: v[ids] for k, v in tab.items() if k not in ("sgn", "hp")}
        A, B, Tw = g["A"][:, None, :], g["B"][:, None, :], g["Tw"][:, None, :]
        ddx = px - g["xa"][:, None]
        ddy = py - g["ya"][:, None]
        # p = k x l in the affine form of raster.hip eval_hit: dx A + dy B + (0, 0, Pz), its fused multiply-adds
        pxc = _fma(ddx, A[..., 0], ddy * B[..., 0])
        pyc = _fma(ddx, A[..., 1], ddy * B[..., 1])
        pzc = _fma(ddy, B[..., 2], _fma(ddx, A[..., 2], g["Pz"][:, None]))
        if tab64 is not None and bool(tab64["hp"][ids].any()):
            # raster.hip hit_p_hp: dx, dy and p of a near-edge-on splat's pairs from its fp64 record, rounded once
            hm = tab64["hp"][ids][:, None]
            x64 = tab64["xa"][ids][:, None]
            y64 = tab64["ya"][ids][:, None]
            A64, B64 = tab64["A"][ids][:, None, :], tab64["B"][ids][:, None, :]
            dx64 = px.double() - x64
            dy64 = py.double() - y64
            if HP_SUM32:
                p32 = _HpPoint.apply(dx64.detach(), dy64.detach(), A64, B64, tab64["Pz"][ids][:, None])
                p64 = [p32[..., 0], p32[..., 1], p32[..., 2]]
            else:
                p64 = [dx64 * A64[..., 0] + dy64 * B64[..., 0], dx64 * A64[..., 1] + dy64 * B64[..., 1],
                       dy64 * B64[..., 2] + (dx64 * A64[..., 2] + tab64["Pz"][ids][:, None])]
            pxc = torch.where(hm, p64[0].float(), pxc)
            pyc = torch.where(hm, p64[1].float(), pyc)
            pzc = torch.where(hm, p64[2].float(), pzc)
        if CAPTURE is not None and decisions is not None:
            src = tab64 if tab64 is not None else tab
            rec = dict(ids=ids, pxi=pxi, pyi=pyi, dx32=ddx.detach(), dy32=ddy.detach(),
                       dx64=(px.double() - src["xa"][ids][:, None].double()).detach(),
                       dy64=(py.double() - src["ya"][ids][:, None].double()).detach(),
                       hp=(tab64["hp"][ids] if tab64 is not None else torch.zeros(K, dtype=torch.bool)))
            for nm, tt in (("gx", pxc), ("gy", pyc), ("gz", pzc)):
                if tt.requires_grad:
                    tt.register_hook(lambda gr, nm=nm, rec=rec: rec.__setitem__(nm, gr.detach().clone()))
            CAPTURE.append(rec)
        else:
            rec = None
        if decisions is None:
            nz = pzc != 0
        else:
            d = decisions["tiles"][t]
            nz = d["nz"]
        pzs = torch.where(nz, pzc, torch.ones_like(pzc))
        ipz = _div(_c(1.0, dtype), pzs)  # raster.hip eval_hit: one reciprocal, two products
        u = pxc * ipz
        v = pyc * ipz
        rho3 = _fma(u, u, v * v)
        dx = g["xy"][:, None, 0] - px
        dy = g["xy"][:, None, 1] - py
        rho2 = fis * _fma(dx, dx, dy * dy)
        if decisions is None:
            use3 = (rho3 <= rho2) if aa else torch.ones_like(rho3, dtype=torch.bool)
        else:
            use3 = d["use3"]
        rho = torch.where(use3, rho3, rho2)
        zz = torch.where(use3, _fma(u, Tw[..., 0], _fma(v, Tw[..., 1], Tw[..., 2])), Tw[..., 2].expand_as(u))
        G = torch.exp(-0.5 * rho)
        a_raw = g["opac"][:, None] * G
        if decisions is None:
            aclamp = a_raw >= amax  # fminf(0.99, a) picks 0.99 iff a >= 0.99 (a > 0.99 differs only at ==)
            alpha = torch.minimum(a_raw, amax)
            valid = nz & (zz >= near) & (alpha >= amin)
            a_eff = torch.where(valid, alpha, torch.zeros_like(alpha))
            Tafter = torch.cumprod(1.0 - a_eff, dim=0)
            stop = valid & (Tafter < tmin)
            any_stop = stop.any(0)
            first = torch.where(any_stop, stop.float().argmax(0), torch.full((P,), K, dtype=torch.int64))
            kidx = torch.arange(K)[:, None]
            incl = valid & (kidx < first[None, :])
            # decision margins (test support): the relative distance of every threshold test the GPU repeats in
            # fp32 (alpha >= 1/255, z >= near, T (1 - alpha) < 1e-4, rho3 <= rho2) from its threshold, over the
            # pairs the traversal reaches.  The GPU evaluates exp and 1 / p.z with the hardware v_exp_f32 /
            # v_rcp_f32 (raster.hip eval_hit), a few ulps from this restatement, so alpha can differ by ~5e-7
            # relative and 1 - alpha by alpha / (1 - alpha) times that: the termination margin is measured in
            # those units
            big = torch.full_like(alpha, float("inf"))
            m_a = (alpha - amin).abs() / amin
            m_z = (zz - near).abs() / near
            sens = torch.clamp(alpha / torch.clamp(1.0 - alpha, min=1e-6), min=1.0)
            m_t = torch.where(valid, (Tafter - tmin).abs() / tmin / sens, big)
            m_u = (rho3 - rho2).abs() / torch.clamp(rho2, min=1e-30) if aa else big
            m_all = torch.minimum(torch.minimum(m_a, m_z), torch.minimum(m_t, m_u))
            margin = torch.where(nz & (kidx <= first[None, :]), m_all, big).min(0).values.float()
        else:
            aclamp = d["aclamp"]
            incl = d["incl"]
            alpha = torch.where(aclamp, amax.expand_as(a_raw), a_raw)
        a_inc = torch.where(incl, alpha, torch.zeros_like(alpha))
        one_m = 1.0 - a_inc
        Tcum = torch.cumprod(one_m, dim=0)
        Tbefore = torch.cat([torch.ones(1, P, dtype=dtype), Tcum[:-1]], 0)
        w = a_inc * Tbefore
        Tfin = Tcum[-1]
        # texture
        h_ = tdims[ids, 0][:, None]
        w_ = tdims[ids, 1][:, None]
        off = tdims[ids, 2][:, None]
        has_tex = (h_ * w_) > 0
        # raster.hip tex_coords: the sample point in texel units from the prescaled affine
        xr = _fma(u, g["auu"][:, None], _fma(v, g["auv"][:, None], g["tu0"][:, None]))
        yr = _fma(u, g["avu"][:, None], _fma(v, g["avv"][:, None], g["tv0"][:, None]))
        hf = h_.to(dtype)
        wf = w_.to(dtype)
        if decisions is None:
            x = torch.minimum(torch.maximum(xr, c(0.0)), hf - 1.0)
            y = torch.minimum(torch.maximum(yr, c(0.0)), wf - 1.0)
            in_u = (xr > 0) & (xr < hf - 1.0)
            in_v = (yr > 0) & (yr < wf - 1.0)
            i0 = torch.where(has_tex, x, torch.zeros_like(x)).clamp(min=0).to(torch.int64)
            j0 = torch.where(has_tex, y, torch.zeros_like(y)).clamp(min=0).to(torch.int64)
        else:
            in_u, in_v, i0, j0 = d["in_u"], d["in_v"], d["i0"], d["j0"]
            x = torch.where(in_u, xr, torch.minimum(torch.maximum(xr, c(0.0)), hf - 1.0).detach())
            y = torch.where(in_v, yr, torch.minimum(torch.maximum(yr, c(0.0)), wf - 1.0).detach())
        hm1 = torch.clamp(h_ - 1, min=0)
        wm1 = torch.clamp(w_ - 1, min=0)
        i1 = torch.minimum(i0 + 1, hm1)
        j1 = torch.minimum(j0 + 1, wm1)
        ax = x - i0.to(dtype)
        ay = y - j0.to(dtype)
        texm = has_tex & incl
        T_n = max(tex.shape[0], 1)

        def fetch(ii, jj):
            idx = torch.where(texm, off + ii * w_ + jj, torch.zeros_like(ii)).clamp(0, T_n - 1)
            if tex.shape[0] == 0:
                return torch.zeros(K, P, C, dtype=dtype)
            return tex[idx.reshape(-1)].reshape(K, P, C)

        v00, v01, v10, v11 = fetch(i0, j0), fetch(i0, j1), fetch(i1, j0), fetch(i1, j1)
        axc, ayc = ax[..., None], ay[..., None]
        top = (1.0 - ayc) * v00 + ayc * v01
        bot = (1.0 - ayc) * v10 + ayc * v11
        tval = (1.0 - axc) * top + axc * bot
        tval = torch.where(texm[..., None], tval, torch.zeros_like(tval))
        wz = torch.where(incl, w, torch.zeros_like(w))
        img = (wz[..., None] * g["rgb"][:, None, :]).sum(0) + Tfin[:, None] * bg[None, :]
        texo = (wz[..., None] * tval).sum(0)
        zsafe = torch.where(incl, zz, torch.ones_like(zz))
        depth = (wz * zsafe).sum(0)
        normal = (wz[..., None] * g["nrm"][:, None, :]).sum(0)
        if dreg:
            m = far * (1.0 - _div(near, zsafe))
            mw = m * wz
            m2w = m * m * wz
            M1b = torch.cumsum(mw, 0) - mw
            M2b = torch.cumsum(m2w, 0) - m2w
            A = 1.0 - Tbefore
            reg = (((m * m * A + M2b) - 2.0 * m * M1b) * wz).sum(0)
            M1 = mw.sum(0)
            M2 = m2w.sum(0)
        else:
            reg = torch.zeros(P, dtype=dtype)
            M1 = torch.zeros(P, dtype=dtype)
            M2 = torch.zeros(P, dtype=dtype)
        if edit is not None:  # texture_edit (raster.hip texture_edit_kernel): fp32 per-pair products, fp64 sums
            pid = torch.from_numpy(pyi * W + pxi)
            erg = edit["rgb"].reshape(-1, 3)[pid].to(dtype)
            ea = edit["a"].reshape(-1)[pid].to(dtype)
            sel = texm & (zz >= edit["lo"].reshape(-1)[pid].to(dtype)[None, :]) & \
                (zz <= edit["hi"].reshape(-1)[pid].to(dtype)[None, :])
            wcs = [(1.0 - ax) * (1.0 - ay), (1.0 - ax) * ay, ax * (1.0 - ay), ax * ay]
            for (ii, jj), wc in zip(((i0, j0), (i0, j1), (i1, j0), (i1, j1)), wcs):
                bw = wc * w
                baw = bw * ea[None, :]
                vals = torch.stack([baw * erg[None, :, 0], baw * erg[None, :, 1], baw * erg[None, :, 2], baw, bw], -1)
                idx = (off + ii * w_ + jj)[sel]
                edit["out"].index_add_(0, idx, vals[sel].to(torch.float64))
        kk = torch.arange(K)[:, None].expand(K, P)
        last = torch.where(incl, kk, torch.full_like(kk, -1)).max(0).values
        if rec is not None:  # (precision analysis: the pair values of this fp32 pass)
            rec.update({k: v.detach().clone() for k, v in dict(
                u=u, v=v, ipz=ipz, use3=use3, zz=zz, G=G, a_raw=a_raw, alpha=alpha, incl=incl, w=w,
                xy=g["xy"], rgb=g["rgb"], nrm=g["nrm"], Tw=g["Tw"], opac=g["opac"], Tfin=Tfin, M1=M1, M2=M2,
                last=last).items()})
            rec["aclamp"] = aclamp.clone()
            rec["t"] = t
        rows["img"].append(img); rows["depth"].append(depth); rows["reg"].append(reg)
        rows["T"].append(Tfin); rows["tex"].append(texo); rows["normal"].append(normal)
        rows["M1"].append(M1); rows["M2"].append(M2)
        last_all.append(last)
        margin_all.append(margin if decisions is None else torch.full((P,), float("inf")))
        if new_dec is not None:
            new_dec["tiles"][t] = dict(nz=nz, use3=use3, aclamp=aclamp, incl=incl, in_u=in_u, in_v=in_v,
                                       i0=i0, j0=j0)

    Np = H * W
    out = {}
    if pix_idx:
        idx = torch.cat(pix_idx)
        order = torch.argsort(idx)

        def assemble(name, width):
            x = torch.cat(rows[name], 0)[order]
            return x.reshape(H, W, width) if width else x.reshape(H, W)

        normal = assemble("normal", 3)
        if inp.settings & SETTING_EVAL_NORMAL:  # raster.hip raster_fwd_kernel: unit normal, 0 where none accumulated
            n2 = (normal[..., 0] * normal[..., 0] + normal[..., 1] * normal[..., 1]) + normal[..., 2] * normal[..., 2]
            inv = torch.where(n2 > 0, _div(_c(1.0, n2.dtype), _sqrt(torch.where(n2 > 0, n2, torch.ones_like(n2)))),
                              torch.zeros_like(n2))
            normal = normal * inv[..., None]
        out = dict(img=assemble("img", 3), depth=assemble("depth", 0), reg=assemble("reg", 0),
                   alpha=1.0 - assemble("T", 0), tex=assemble("tex", C), normal=normal,
                   T_final=assemble("T", 0), M1=assemble("M1", 0), M2=assemble("M2", 0))
        last_img = torch.cat(last_all)[order].reshape(H, W)
        margin_img = torch.cat(margin_all)[order].reshape(H, W)
    else:
        last_img = torch.full((H, W), -1)
        margin_img = torch.full((H, W), float("inf"))
    assert Np == H * W
    res = dict(out=out, last=last_img, margin=margin_img)
    if new_dec is not None:
        res["decisions"] = new_dec
    return res


def texture_edit(inp: RasterInputs, edit_rgb, edit_alpha, depth_lo, depth_hi, bins=None):
    """raster.hip:texture_edit_kernel (gstex.py:579-606).  The fp32 decision pass of the forward
    (same inclusion, weights w = alpha * T, hit depth, texel cell) with the stroke scattered to the
    texels: out[texel] += b * w * (a*rgb, a, 1) for pairs with depth_lo <= z <= depth_hi.  Per-pair
    products in fp32 (the kernel's operation order), sums in fp64; returns (T, 5) float64."""
    cam = inp.cam
    if bins is None:
        bins = bin_and_sort(inp.centers, inp.extents, inp.depths, cam.H, cam.W, cam.block)
    n_tex = inp.texture.shape[0]
    edit = dict(rgb=edit_rgb, a=edit_alpha, lo=depth_lo, hi=depth_hi,
                out=torch.zeros((n_tex, 5), dtype=torch.float64))
    from dataclasses import replace
    _render(replace(inp, hp=False), F32, bins[1], bins[2], None, edit=edit)  # (its records carry no hp rows)
    return edit["out"]


# ----------------------------------------------------------------------------------------
# spherical harmonics and texture resampling (sh_texture.hip)
# ----------------------------------------------------------------------------------------
SH_C0 = np.float32(0.28209479177387814)
SH_C1 = np.float32(0.4886025119029199)
SH_C2 = [np.float32(v) for v in (1.0925484305920792, -1.0925484305920792, 0.31539156525252005,
                                 -1.0925484305920792, 0.5462742152960396)]
SH_C3 = [np.float32(v) for v in (-0.5900435899266435, 2.890611442640554, -0.4570457994644658,
                                 0.3731763325901154, -0.4570457994644658, 1.445305721320277,
                                 -0.5900435899266435)]
SH_C4 = [np.float32(v) for v in (2.5033429417967046, -1.7701307697799304, 0.9461746957575601,
                                 -0.6690465435572892, 0.10578554691520431, -0.6690465435572892,
                                 0.47308734787878004, -1.7701307697799304, 0.6258357354491761)]


def num_sh_bases(degree: int) -> int:
    return (degree + 1) ** 2


def sh_basis(degree, dirs, dtype=F32):
    """sh_texture.hip:sh_basis (gsplat-0.1 real SH basis)."""
    c = lambda v: _c(v, dtype)  # noqa: E731
    d = dirs.to(dtype)
    n = d.shape[0]
    b = [c(SH_C0).expand(n)]
    if degree < 1:
        return torch.stack(b, -1)
    x, y, z = d.unbind(-1)
    nrm = _sqrt((x * x + y * y) + z * z)
    x, y, z = _div(x, nrm), _div(y, nrm), _div(z, nrm)
    b += [-c(SH_C1) * y, c(SH_C1) * z, -c(SH_C1) * x]
    if degree >= 2:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        b += [c(SH_C2[0]) * xy, c(SH_C2[1]) * yz, c(SH_C2[2]) * ((2.0 * zz - xx) - yy), c(SH_C2[3]) * xz,
              c(SH_C2[4]) * (xx - yy)]
    if degree >= 3:
        b += [c(SH_C3[0]) * y * (3.0 * xx - yy), c(SH_C3[1]) * xy * z, c(SH_C3[2]) * y * ((4.0 * zz - xx) - yy),
              c(SH_C3[3]) * z * ((2.0 * zz - 3.0 * xx) - 3.0 * yy), c(SH_C3[4]) * x * ((4.0 * zz - xx) - yy),
              c(SH_C3[5]) * z * (xx - yy), c(SH_C3[6]) * x * (xx - 3.0 * yy)]
    if degree >= 4:
        b += [c(SH_C4[0]) * xy * (xx - yy), c(SH_C4[1]) * yz * (3.0 * xx - yy), c(SH_C4[2]) * xy * (7.0 * zz - 1.0),
              c(SH_C4[3]) * yz * (7.0 * zz - 3.0), c(SH_C4[4]) * (zz * (35.0 * zz - 30.0) + 3.0),
              c(SH_C4[5]) * xz * (7.0 * zz - 3.0), c(SH_C4[6]) * (xx - yy) * (7.0 * zz - 1.0),
              c(SH_C4[7]) * xz * (xx - 3.0 * yy), c(SH_C4[8]) * (xx * (xx - 3.0 * yy) - yy * (3.0 * xx - yy))]
    return torch.stack(b, -1)


def spherical_harmonics(degree, viewdirs, coeffs, dtype=F32):
    """gstex_cuda.sh.spherical_harmonics (gstex.py:1109): sum_k basis_k * coeffs[:,k,:], no +0.5."""
    b = sh_basis(degree, viewdirs, dtype)
    nb = num_sh_bases(degree)
    cf = coeffs.to(dtype)[:, :nb, :]
    out = torch.zeros(cf.shape[0], 3, dtype=dtype)
    for k in range(nb):  # sequential accumulation like the kernel
        out = out + b[:, k : k + 1] * cf[:, k, :]
    return out


def texture_sample(query_dims, texture, uv, dtype=F32):
    """gstex_cuda.texture_sample.texture_sample (jagged_texture.py:138): bilinear resample of each
    query's texel block (corner-aligned, clamp-to-edge; gstex_common.h:bilerp_coords)."""
    qd = query_dims.long()
    h, w, off = qd[:, 0], qd[:, 1], qd[:, 2]
    tex = texture.to(dtype)
    C = tex.shape[1]
    has = (h * w) > 0
    hf, wf = h.to(dtype), w.to(dtype)
    u = uv[:, 0].to(dtype)
    v = uv[:, 1].to(dtype)
    x = torch.minimum(torch.maximum(u * hf, _c(0.0, dtype)), hf - 1.0)
    y = torch.minimum(torch.maximum(v * wf, _c(0.0, dtype)), wf - 1.0)
    i0 = torch.where(has, x, torch.zeros_like(x)).clamp(min=0).long()
    j0 = torch.where(has, y, torch.zeros_like(y)).clamp(min=0).long()
    i1 = torch.minimum(i0 + 1, (h - 1).clamp(min=0))
    j1 = torch.minimum(j0 + 1, (w - 1).clamp(min=0))
    ax = (x - i0.to(dtype))[:, None]
    ay = (y - j0.to(dtype))[:, None]
    Tn = max(tex.shape[0], 1)

    def f(ii, jj):
        idx = torch.where(has, off + ii * w + jj, torch.zeros_like(ii)).clamp(0, Tn - 1)
        return tex[idx] if tex.shape[0] else torch.zeros(qd.shape[0], C, dtype=dtype)

    top = (1.0 - ay) * f(i0, j0) + ay * f(i0, j1)
    bot = (1.0 - ay) * f(i1, j0) + ay * f(i1, j1)
    out = (1.0 - ax) * top + ax * bot
    return torch.where(has[:, None], out, torch.zeros_like(out))
