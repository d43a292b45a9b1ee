"""Host-side mirror of GStex's per-splat texture charting (the data format the rasterizer reads).

* texture_dims_to_int_coords / texture_dims_to_query  <- models/jagged_texture.py:10-34
* build_charts                                        <- models/gstex.py:841-888
* get_uv_mapping                                      <- models/gstex.py:975-990
* SH2RGB / RGB2SH / random_quat_tensor                <- models/gstex.py:68-99

Pinned against goldens generated from the reference functions (tests/golden/make_golden.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from gstex_cuda._torch_impl import quat_to_rotmat

SH_C0 = 0.28209479177387814


def SH2RGB(sh):
    return sh * SH_C0 + 0.5


def RGB2SH(rgb):
    return (rgb - 0.5) / SH_C0


def random_quat_tensor(N: int, generator: torch.Generator | None = None) -> torch.Tensor:
    """Uniform random unit quaternions (gstex.py:68-83)."""
    u = torch.rand(N, generator=generator)
    v = torch.rand(N, generator=generator)
    w = torch.rand(N, generator=generator)
    return torch.stack(
        [
            torch.sqrt(1 - u) * torch.sin(2 * math.pi * v),
            torch.sqrt(1 - u) * torch.cos(2 * math.pi * v),
            torch.sqrt(u) * torch.sin(2 * math.pi * w),
            torch.sqrt(u) * torch.cos(2 * math.pi * w),
        ],
        dim=-1,
    )


def _ids(texture_dims):
    idxs = torch.arange(texture_dims.shape[0], dtype=torch.int64, device=texture_dims.device)
    hws = (texture_dims[:, 0] * texture_dims[:, 1]).long()
    ids = torch.repeat_interleave(idxs, hws, dim=0)
    return ids, int(hws.sum().item())


def texture_dims_to_int_coords(texture_dims):
    """Per texel: owning splat id and integer (i, j) inside its h x w block."""
    ids, total = _ids(texture_dims)
    q = texture_dims[ids, :].long()
    local = torch.arange(total, dtype=torch.int64, device=texture_dims.device) - q[:, 2]
    return ids, torch.stack([local // q[:, 1], local % q[:, 1]], dim=-1)


def texture_dims_to_query(texture_dims):
    """Per texel: owning splat id and its texel-centre uv = (i/h, j/w)."""
    ids, total = _ids(texture_dims)
    q = texture_dims[ids, :].long()
    local = torch.arange(total, dtype=torch.int64, device=texture_dims.device) - q[:, 2]
    uu = (local // q[:, 1]).float() / q[:, 0].float()
    vv = (local % q[:, 1]).float() / q[:, 1].float()
    return ids, torch.stack([uu, vv], dim=-1)


def build_charts(log_scales: torch.Tensor, pixel_num: float, sigma_factor: float = 3.0, max_iter: int = 30):
    """Texel budget allocation (gstex.py:841-888).

    Bisection on the texel size `pixel_scale` so that sum(ceil(sf*e^s0/ps) * ceil(sf*e^s1/ps)) is
    within 0.1 % of pixel_num.  Returns (texture_dims int32 (N,3) = [h, w, offset], mappings (N,2),
    pixel_scale float).  pixel_num must be > 0 (the reference divides by it, gstex.py:857)."""
    if pixel_num <= 0:
        raise ZeroDivisionError("build_charts: pixel_num must be > 0 (2DGS mode uses all-zero texture_dims)")
    with torch.no_grad():
        length0 = torch.exp(log_scales[:, 0])
        length1 = torch.exp(log_scales[:, 1])

        def get_score(x):
            return torch.sum(torch.ceil(sigma_factor * length0 / x) * torch.ceil(sigma_factor * length1 / x)).item()

        adjustments = torch.ones_like(length0)
        adjustments = torch.sqrt(adjustments**2 / torch.mean(adjustments**2))
        lo = 10.0
        hi = np.sqrt(torch.sum(sigma_factor * sigma_factor * length0 * length1 * (adjustments**2)).item() / pixel_num)
        mid = 0.5 * (lo + hi)
        score = get_score(mid)
        it = 0
        tol = 1e-3
        while score < (1 - tol) * pixel_num or score > (1 + tol) * pixel_num:
            if score < (1 - tol) * pixel_num:
                lo = mid
            else:
                hi = mid
            mid = 0.5 * (lo + hi)
            score = get_score(mid / adjustments)
            it += 1
            if it > max_iter:
                break
        pixel_scales = mid / adjustments
        n = log_scales.shape[0]
        dims = torch.zeros(n, 3, dtype=torch.int32, device=log_scales.device)
        dims[:, 0] = torch.ceil(sigma_factor * length0 / pixel_scales).int()
        dims[:, 1] = torch.ceil(sigma_factor * length1 / pixel_scales).int()
        hws = dims[:, 0] * dims[:, 1]
        dims[:, 2] = torch.cumsum(hws, dim=0) - hws
        mappings = torch.stack([1 / (2.0 * sigma_factor * length0), 1 / (2.0 * sigma_factor * length1)], -1)
    return dims, mappings, float(mid)


def get_uv_mapping(quats: torch.Tensor, mappings: torch.Tensor):
    """(uv0 (N,1,2), umap (N,1,3), vmap (N,1,3)), all detached (gstex.py:975-990)."""
    uv0 = 0.5 * torch.ones((quats.shape[0], 2), device=quats.device, dtype=quats.dtype)
    Rs = quat_to_rotmat(quats.detach())
    umap = mappings[:, 0, None].detach() * Rs[:, :, 0].detach()
    vmap = mappings[:, 1, None].detach() * Rs[:, :, 1].detach()
    return uv0.unsqueeze(1), umap.unsqueeze(1), vmap.unsqueeze(1)
