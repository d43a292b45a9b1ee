"""Fused splat activations and DC-free SH colour (``gstex_activate_*``, ``gstex_sh_rest_*``).

``activate(means, quats, log_scales, opacity_logits, mappings, campos)`` returns what
GStexModel.get_outputs derives from the stored parameters each step (gstex.py:1059-1066, 975-990,
1101-1104): normalised quaternions, activated scales (third axis 1e-5 x mean, detached), opacities,
and the detached uv0/umap/vmap frames and SH view directions -- one HIP launch forward, one backward,
instead of ~40 small torch kernels.  ``sh_rest(degree, viewdirs, features_rest)`` is
``spherical_harmonics(degree, viewdirs, cat([0, features_rest]))`` without materialising the cat.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import call, ptr


def _f32c(t, name, shape):
    if t.dtype != torch.float32 or not t.is_cuda or tuple(t.shape) != shape:
        raise ValueError(f"{name}: expected a CUDA float32 tensor of shape {shape}, got {t.dtype} {tuple(t.shape)}")
    return t.contiguous()


class _Activate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means, quats, log_scales, opacity_logits, mappings, campos):
        n = means.shape[0]
        means = _f32c(means.detach(), "means", (n, 3))
        quats = _f32c(quats.detach(), "quats", (n, 4))
        log_scales = _f32c(log_scales.detach(), "scales", (n, 3))
        logits = _f32c(opacity_logits.detach(), "opacities", (n, 1))
        mp = mappings.detach()
        if mp.dim() != 2 or mp.shape[0] != n or mp.shape[1] < 2 or mp.dtype != torch.float32:
            raise ValueError("mappings: expected float32 (N, >=2)")
        mp = mp.contiguous()
        campos = _f32c(campos.detach().reshape(3), "campos", (3,))
        f = dict(device=means.device, dtype=torch.float32)
        qn = torch.empty((n, 4), **f)
        sc = torch.empty((n, 3), **f)
        op = torch.empty((n, 1), **f)
        uv0 = torch.empty((n, 1, 2), **f)
        umap = torch.empty((n, 1, 3), **f)
        vmap = torch.empty((n, 1, 3), **f)
        vd = torch.empty((n, 3), **f)
        call("gstex_activate_fwd", n, ptr(means), ptr(quats), ptr(log_scales), ptr(logits), ptr(mp), mp.shape[1],
             ptr(campos), ptr(qn), ptr(sc), ptr(op), ptr(uv0), ptr(umap), ptr(vmap), ptr(vd),
             _lib.stream_of(means.device))
        ctx.save_for_backward(quats, log_scales, op)
        ctx.mark_non_differentiable(uv0, umap, vmap, vd)
        ctx.set_materialize_grads(False)  # no zero tensors for the detached outputs; the kernel reads NULL as 0
        return qn, sc, op, uv0, umap, vmap, vd

    @staticmethod
    def backward(ctx, g_qn, g_sc, g_op, *_):
        quats, log_scales, op = ctx.saved_tensors
        n = quats.shape[0]
        nq, ns, no = ctx.needs_input_grad[1], ctx.needs_input_grad[2], ctx.needs_input_grad[3]
        v_q = torch.empty_like(quats) if nq else None
        v_s = torch.empty_like(log_scales) if ns else None
        v_o = torch.empty_like(op) if no else None
        c = lambda t: None if t is None else t.contiguous()  # noqa: E731
        call("gstex_activate_bwd", n, ptr(quats), ptr(log_scales), ptr(op), ptr(c(g_qn)), ptr(c(g_sc)), ptr(c(g_op)),
             ptr(v_q), ptr(v_s), ptr(v_o), _lib.stream_of(quats.device))
        return None, v_q, v_s, v_o, None, None


def activate(means, quats, log_scales, opacity_logits, mappings, campos):
    """-> (quats_n, scales, opacities, uv0, umap, vmap, viewdirs); see the module docstring."""
    return _Activate.apply(means, quats, log_scales, opacity_logits, mappings, campos)


class _SHRest(torch.autograd.Function):
    @staticmethod
    def forward(ctx, degree, viewdirs, rest):
        n = viewdirs.shape[0]
        vd = _f32c(viewdirs.detach(), "viewdirs", (n, 3))
        if rest.dim() != 3 or rest.shape[0] != n or rest.shape[2] != 3 or rest.dtype != torch.float32:
            raise ValueError("features_rest: expected float32 (N, K, 3)")
        r = rest.detach().contiguous()
        out = torch.empty((n, 3), device=vd.device, dtype=torch.float32)
        call("gstex_sh_rest_fwd", n, int(degree), r.shape[1], ptr(vd), ptr(r), ptr(out), _lib.stream_of(vd.device))
        ctx.save_for_backward(vd)
        ctx.degree, ctx.K = int(degree), r.shape[1]
        return out

    @staticmethod
    def backward(ctx, g):
        (vd,) = ctx.saved_tensors
        n = vd.shape[0]
        v = torch.empty((n, ctx.K, 3), device=vd.device, dtype=torch.float32)
        call("gstex_sh_rest_bwd", n, ctx.degree, ctx.K, ptr(vd), ptr(g.contiguous()), ptr(v), _lib.stream_of(vd.device))
        return None, None, v


def sh_rest(degree: int, viewdirs, features_rest):
    return _SHRest.apply(degree, viewdirs, features_rest)
