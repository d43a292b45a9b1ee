"""Fused GStex photometric loss (``gstex_loss_fwd`` / ``gstex_loss_bwd``).

``photometric_loss(img, tex, alpha, background, gt)`` is the reference's training loss on the raw
rasterizer outputs: the background composite and clamp (gstex.py:1204-1205) followed by
``0.8 * L1 + 0.2 * (1 - SSIM)`` (gstex.py:1301-1322, pytorch_msssim SSIM, 11-tap sigma-1.5 window,
valid filtering).  One forward launch (+ a one-workgroup reduction) and one backward launch replace
the ~40 elementwise kernels and four GEMMs the same expression costs in eager PyTorch.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import call, ptr

_WINDOWS: dict = {}
_CWIN = None


def _cwin():
    """The 11-tap window as the C array the loss kernels take (built once: no per-step tensor-to-list work)."""
    global _CWIN
    if _CWIN is None:
        _CWIN = (ctypes.c_float * 11)(*(float(x) for x in gaussian_window().numpy()))
    return _CWIN


def gaussian_window(size: int = 11, sigma: float = 1.5) -> torch.Tensor:
    """pytorch_msssim._fspecial_gauss_1d, evaluated in fp32 on the CPU."""
    key = (size, sigma)
    w = _WINDOWS.get(key)
    if w is None:
        coords = torch.arange(size, dtype=torch.float32) - size // 2
        g = torch.exp(-(coords**2) / (2 * sigma**2))
        w = (g / g.sum()).contiguous()
        _WINDOWS[key] = w
    return w


def _check(img, tex, alpha, background, gt):
    H, W = alpha.shape
    for name, t, shape in (("img", img, (H, W, 3)), ("alpha", alpha, (H, W)), ("gt", gt, (H, W, 3)),
                           ("background", background, (3,))):
        if tuple(t.shape) != shape or t.dtype != torch.float32 or not t.is_cuda:
            raise ValueError(f"photometric_loss: {name} must be a CUDA fp32 tensor of shape {shape}")
    if tex.dim() != 3 or tuple(tex.shape[:2]) != (H, W) or not 3 <= tex.shape[2] <= 8 or tex.dtype != torch.float32:
        raise ValueError("photometric_loss: tex must be CUDA fp32 (H, W, C) with 3 <= C <= 8")
    if H <= 10 or W <= 10:
        raise ValueError("photometric_loss: the image must be larger than the 11-tap SSIM window")


class _PhotometricLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, tex, alpha, background, gt, ssim_lambda):
        _check(img, tex, alpha, background, gt)
        img, tex, alpha, background, gt = (t.detach().contiguous() for t in (img, tex, alpha, background, gt))
        H, W = alpha.shape
        C = tex.shape[2]
        cwin = _cwin()
        ws = torch.empty((int(_lib.load().gstex_loss_workspace_size(H, W)),), device=img.device, dtype=torch.uint8)
        out = torch.empty((3,), device=img.device, dtype=torch.float32)
        rgb = torch.empty((H, W, 3), device=img.device, dtype=torch.float32)
        st = _lib.stream_of(img.device)
        call("gstex_loss_fwd", H, W, C, ptr(img), ptr(tex), ptr(alpha), ptr(background), ptr(gt), cwin,
             float(ssim_lambda), ptr(rgb), ptr(out), ptr(ws), ws.numel(), st)
        ctx.save_for_backward(img, tex, alpha, background, gt, ws)
        ctx.ssim_lambda = float(ssim_lambda)
        ctx.mark_non_differentiable(rgb)
        ctx.set_materialize_grads(False)  # rgb's (always unused) gradient stays None, no zero image
        return out[0], rgb  # out[1:] = (L1, SSIM) stay readable through the base tensor

    @staticmethod
    def backward(ctx, g_loss, g_rgb):
        if g_loss is None:
            return None, None, None, None, None, None
        img, tex, alpha, background, gt, ws = ctx.saved_tensors
        H, W = alpha.shape
        C = tex.shape[2]
        cwin = _cwin()
        d_img = torch.empty_like(img)
        d_tex = torch.empty_like(tex)
        d_alpha = torch.empty_like(alpha)
        g = g_loss.detach().to(torch.float32).contiguous()
        call("gstex_loss_bwd", H, W, C, ptr(img), ptr(tex), ptr(alpha), ptr(background), ptr(gt), cwin,
             ctx.ssim_lambda, g.data_ptr(), ptr(d_img), ptr(d_tex), ptr(d_alpha), ptr(ws), ws.numel(),
             _lib.stream_of(img.device))
        return d_img, d_tex, d_alpha, None, None, None


def photometric_loss(img, tex, alpha, background, gt, ssim_lambda: float = 0.2):
    """Returns (loss, rgb): loss is the differentiable 0-dim training loss, rgb the composited image."""
    return _PhotometricLoss.apply(img, tex, alpha, background, gt, ssim_lambda)


# ---------------------------------------------------------------------------------------------------------------
# geometry regularisers of get_loss_dict (gstex.py:1313-1317), for a trainer with depth / normal renders
# ---------------------------------------------------------------------------------------------------------------
def depths_to_points(depth: torch.Tensor, viewmat: torch.Tensor, c2w: torch.Tensor, fx: float, fy: float, cx: float,
                     cy: float) -> torch.Tensor:
    """World-space points (H, W, 3) of a rendered depth map, as the reference's depths_to_points
    (gstex.py:122-149): pixel (i, j) looks along the unit world ray of camera direction ((j - cx + 0.5) / fx,
    (i - cy + 0.5) / fy, 1); the depth is view-space z ("don't use view depth", :145-146), so the distance along
    the ray is depth / (the ray's view-space z component)."""
    H, W = depth.shape[0], depth.shape[1]
    dev, f = depth.device, torch.float32
    rows = torch.arange(H, device=dev, dtype=f)[:, None].expand(H, W)
    cols = torch.arange(W, device=dev, dtype=f)[None, :].expand(H, W)
    cam_dir = torch.stack([(cols - cx + 0.5) / fx, (rows - cy + 0.5) / fy, torch.ones_like(rows)], dim=-1)
    world_dir = cam_dir @ c2w[:3, :3].to(f).T
    world_dir = world_dir / (world_dir.norm(dim=-1, keepdim=True) + 1e-9)
    view_z = world_dir @ viewmat[2, :3].to(f)
    dist = depth.reshape(H, W) / view_z
    return c2w[:3, 3].to(f) + dist[..., None] * world_dir


def depth_to_normal(depth: torch.Tensor, viewmat: torch.Tensor, c2w: torch.Tensor, fx: float, fy: float, cx: float,
                    cy: float) -> torch.Tensor:
    """Normals (H, W, 3) estimated from a depth map, as the reference's depth_to_normal (gstex.py:151-161): the unit
    cross product of the central differences of depths_to_points down the rows and along the columns; the one-pixel
    border is zero."""
    p = depths_to_points(depth, viewmat, c2w, fx, fy, cx, cy)
    d_rows = p[2:, 1:-1] - p[:-2, 1:-1]
    d_cols = p[1:-1, 2:] - p[1:-1, :-2]
    out = torch.zeros_like(p)
    out[1:-1, 1:-1] = torch.nn.functional.normalize(torch.linalg.cross(d_rows, d_cols, dim=-1), dim=-1)
    return out


def scheduled(value, step: int) -> float:
    """A loss weight as get_loss_dict reads it (gstex.py:1304-1311): a number, or [before, after, switch_step]."""
    if isinstance(value, (int, float)):
        return float(value)
    return float(value[1] if step >= value[2] else value[0])


def geometry_loss(alpha: torch.Tensor, normal: torch.Tensor, estimated_normal: torch.Tensor, reg: torch.Tensor,
                  lambda_normal: float, lambda_reg: float) -> torch.Tensor:
    """normal_loss + reg_loss of get_loss_dict (gstex.py:1316-1317): lambda_normal * mean(alpha - <n, n_est>) +
    lambda_reg * mean(reg)."""
    loss = alpha.new_zeros(())
    if lambda_normal != 0.0:
        loss = loss + lambda_normal * torch.mean(alpha.reshape(alpha.shape[0], alpha.shape[1])
                                                 - torch.sum(normal * estimated_normal, dim=-1))
    if lambda_reg != 0.0:
        loss = loss + lambda_reg * torch.mean(reg)
    return loss
