"""Synthetic scenes and cameras: random-init splats + charted texels.

Mirrors the reference's random initialisation (gstex.py:276-300: uniform cube means, log of the
mean 3-NN distance for the scales, random unit quaternions, opacity logit(0.1)) and its Blender
camera (fx = 0.5 W / tan(0.5 * 0.6911112), blender_dataparser.py:77-78) on a radius-4.0311 sphere
with the y/z flip of gstex.py:1031-1041.  Seeded on the CPU generator so every device and the
oracle see identical inputs.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from .charts import SH2RGB, build_charts, get_uv_mapping, random_quat_tensor

BLENDER_FOV = 0.6911112
CAM_RADIUS = 4.0311


def knn_mean_dist(points: np.ndarray, k: int = 3) -> np.ndarray:
    from scipy.spatial import cKDTree

    tree = cKDTree(points)
    d, _ = tree.query(points, k=k + 1)
    return d[:, 1:].mean(-1).astype(np.float32)


def look_at(campos, target=(0.0, 0.0, 0.0), up=(0.0, 0.0, 1.0)):
    """OpenGL c2w looking at target -> (viewmat (3,4), c2w (4,4)) after the y/z flip
    (OpenCV axes) exactly as gstex.py:1031-1042 derives them."""
    campos = np.asarray(campos, np.float64)
    f = np.asarray(target, np.float64) - campos
    f /= np.linalg.norm(f)
    r = np.cross(f, np.asarray(up, np.float64))
    if np.linalg.norm(r) < 1e-8:
        r = np.cross(f, np.array([0.0, 1.0, 0.0]))
    r /= np.linalg.norm(r)
    u = np.cross(r, f)
    R = np.stack([r, u, -f], 1) @ np.diag([1.0, -1.0, -1.0])
    vm = np.eye(4)
    vm[:3, :3] = R.T
    vm[:3, 3] = -R.T @ campos
    c2w = np.linalg.inv(vm)
    return torch.tensor(vm[:3, :], dtype=torch.float32), torch.tensor(c2w, dtype=torch.float32)


@dataclass
class View:
    viewmat: torch.Tensor  # (3,4)
    c2w: torch.Tensor      # (4,4)
    fx: float
    fy: float
    cx: float
    cy: float
    H: int
    W: int

    def to(self, device):
        return View(self.viewmat.to(device), self.c2w.to(device), self.fx, self.fy, self.cx, self.cy, self.H, self.W)

    @property
    def campos(self) -> torch.Tensor:
        """The camera centre c2w[:3, 3] as a contiguous (3,) tensor, made once per view (a per-render copy of the
        strided column was a kernel launch of its own).  The cache is keyed on the c2w tensor's identity, storage and
        version counter, so reassigning c2w or editing it in place recomputes it."""
        key = (id(self.c2w), self.c2w.data_ptr(), self.c2w._version, self.c2w.device)
        hit = self.__dict__.get("_campos")
        if hit is None or hit[0] != key:
            hit = (key, self.c2w[:3, 3].contiguous())
            self.__dict__["_campos"] = hit
        return hit[1]


def sphere_view(index: int, H: int, W: int, n_views: int = 8, radius: float = CAM_RADIUS) -> View:
    """Camera `index` of `n_views` spread over a sphere (golden-angle spiral), Blender intrinsics."""
    i = index % max(n_views, 1)
    zc = 0.6 - 1.2 * (i + 0.5) / max(n_views, 1)
    phi = i * math.pi * (3.0 - math.sqrt(5.0)) + 0.3
    rxy = math.sqrt(max(1.0 - zc * zc, 0.0))
    pos = (radius * rxy * math.cos(phi), radius * rxy * math.sin(phi), radius * zc)
    vm, c2w = look_at(pos)
    fx = 0.5 * W / math.tan(0.5 * BLENDER_FOV)
    fy = 0.5 * H / math.tan(0.5 * BLENDER_FOV) if H != W else fx
    return View(vm, c2w, fx, fy, W / 2.0, H / 2.0, H, W)


@dataclass
class Scene:
    means: torch.Tensor
    log_scales: torch.Tensor
    quats: torch.Tensor
    opacity_logits: torch.Tensor
    features_dc: torch.Tensor
    features_rest: torch.Tensor
    rgbs: torch.Tensor
    texture_dims: torch.Tensor
    mappings: torch.Tensor
    texture: torch.Tensor  # (T, C) in [0,1] (raster-space colours)
    pixel_scale: float

    @property
    def n(self):
        return self.means.shape[0]

    def activated(self):
        """Per-step activations of gstex.py:1059-1066 -> (means, scales, quats, opacities)."""
        quats = self.quats / self.quats.norm(dim=-1, keepdim=True)
        scales = torch.zeros_like(self.log_scales)
        scales[:, :-1] = torch.clamp(torch.exp(self.log_scales[:, :-1]), min=1e-9)
        scales[:, -1] = 1e-5 * torch.mean(scales[:, :-1], dim=-1).detach()
        return self.means, scales, quats, torch.sigmoid(self.opacity_logits)

    def uv_mapping(self):
        return get_uv_mapping(self.quats / self.quats.norm(dim=-1, keepdim=True), self.mappings)

    def to(self, device):
        kw = {k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in self.__dict__.items()}
        return Scene(**kw)


def make_scene(n: int, n_texels: float, channels: int = 3, seed: int = 42, cube: float = 2.0,
               opacity: float | None = 0.1, sh_degree: int = 3) -> Scene:
    """Random-init scene of `n` splats with about `n_texels` texels (0 = 2DGS mode: all dims 0)."""
    g = torch.Generator().manual_seed(seed)
    means = (torch.rand((n, 3), generator=g) - 0.5) * cube
    d = knn_mean_dist(means.numpy(), 3) if n > 3 else np.full(n, 0.05, np.float32)
    log_scales = torch.log(torch.from_numpy(d)[:, None].repeat(1, 3))
    quats = random_quat_tensor(n, generator=g)
    if opacity is None:
        op = 0.05 + 0.9 * torch.rand((n, 1), generator=g)
    else:
        op = torch.full((n, 1), float(opacity))
    opacity_logits = torch.logit(op)
    nb = (sh_degree + 1) ** 2
    features_dc = torch.rand((n, 3), generator=g)
    features_rest = 0.1 * torch.randn((n, nb - 1, 3), generator=g)
    rgbs = torch.rand((n, 3), generator=g)
    if n_texels and n_texels > 0:
        dims, mappings, ps = build_charts(log_scales, float(n_texels))
        T = int((dims[:, 0] * dims[:, 1]).sum().item())
    else:
        dims = torch.zeros((n, 3), dtype=torch.int32)
        mappings = torch.stack([1 / (6.0 * torch.exp(log_scales[:, 0])), 1 / (6.0 * torch.exp(log_scales[:, 1]))], -1)
        ps, T = 0.0, 0
    texture = torch.rand((T, channels), generator=g)
    return Scene(means, log_scales, quats, opacity_logits, features_dc, features_rest, rgbs, dims, mappings, texture,
                 ps)


def texture_from_dc(texture_dc: torch.Tensor, channels: int = 3) -> torch.Tensor:
    """Raster texture from the SH-DC texel parameter (gstex.py:1093-1094,1119)."""
    tex = torch.zeros((texture_dc.shape[0], channels), device=texture_dc.device, dtype=texture_dc.dtype)
    tex[:, 0:3] = SH2RGB(texture_dc)
    return tex
