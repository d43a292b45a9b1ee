"""Fused multi-tensor Adam (``gstex_adam_step``) for the GStex parameter groups.

Drop-in for the reference's ``torch.optim.Adam(params, lr, eps=1e-15)`` per group
(gstex_configs.py:207-244, engine/optimizers.py:158-171): the same update, the same
per-parameter ``state`` ({"step", "exp_avg", "exp_avg_sq"}) and ``param_groups``, so code that resets a
parameter's moments (the rechart, gstex.py:799-826) keeps working.  All parameters of all groups are
updated by one HIP launch (16 tensors per launch) instead of torch's ~7 foreach passes.
"""
from __future__ import annotations

import torch

from . import _lib


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        if lr < 0 or eps < 0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid Adam hyper-parameters lr={lr} betas={betas} eps={eps}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps))

    @torch.no_grad()
    def step(self, closure=None, only=None, skip=None, zero_grad=False, grid=0, grad_scale=1.0, skip_flag=None):
        """The Adam update.  Extensions (not in torch.optim.Adam): `only` / `skip` (sets of id(param)) restrict the
        update to / exclude a set of parameters (so one group can be launched on another stream), and `zero_grad` writes zeros over each
        gradient after reading it (gstex_adam_step_ex, GSTEX_ADAM_ZERO_GRAD); `grid` > 0 caps the launch's
        workgroups (GSTEX_ADAM_GRID: each loops over the chunks), leaving CUs to another stream; `grad_scale` in (0, 1]
        multiplies every gradient as it is read (gstex_adam_step_scaled: a data-parallel step's 1 / world, applied to the
        all-reduced sums -- bit-identical to averaging the buffer first); `skip_flag` (a 1-element device fp32 tensor)
        makes the launch a no-op on the device when the value is non-zero (gstex_adam_step_guarded: the pair-capacity
        guard of the step's renders, ops.PairCapacity) -- the step counts still advance, deliberately: the host learns
        of a skipped step only after the fact (no read-back in the step), so unlike GradScaler-style skipping (which
        does not call step() at all) the next real update applies the bias corrections of step t + 1 to moments last
        updated at step t - 1.  The moments themselves are untouched; the difference is a factor
        (1 - beta^t) / (1 - beta^(t+1)) on each correction, which tends to 1 as t grows (< 1e-3 for beta1 = 0.9 once
        t > 60, for beta2 = 0.999 once t > 7000), and an overflow grows the capacity, so it recurs only if the pair
        total keeps jumping.  The launch goes to the current stream."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        # one launch per (betas, eps, device, stream) family; the GStex groups all share them
        batches: dict = {}
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None or (only is not None and id(p) not in only) or (skip is not None and id(p) in skip):
                    continue
                g = p.grad
                if g.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                if p.dtype != torch.float32 or g.dtype != torch.float32 or not p.is_cuda:
                    raise TypeError("FusedAdam: fp32 CUDA parameters and gradients only")
                if not (p.is_contiguous() and g.is_contiguous()):
                    raise ValueError("FusedAdam: parameters and gradients must be contiguous")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["step"] += 1
                t = st["step"]
                # python-double bias corrections, rounded to fp32 exactly where torch's foreach Adam does
                step_size = group["lr"] / (1.0 - b1 ** t)
                bc2_sqrt = (1.0 - b2 ** t) ** 0.5
                desc = _lib.GstexAdamTensor(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                                            st["exp_avg_sq"].data_ptr(), p.numel(), step_size, bc2_sqrt)
                key = (b1, b2, group["eps"], p.device)
                batches.setdefault(key, []).append(desc)
        self._launch(batches, zero_grad, grid, grad_scale, skip_flag)
        return loss

    @torch.no_grad()
    def step_range(self, p, lo: int, hi: int, first: bool, zero_grad=False, grad_scale=1.0, skip_flag=None):
        """The Adam update of elements [lo, hi) of parameter `p` only: the chunks of one step, launched one by one
        (e.g. each as soon as its slice of an all-reduce has landed, gstex_amd.dist.GradSync), together equal one
        step(only={id(p)}) bit for bit (the update is elementwise).  `first`: the chunk that advances the parameter's
        step count (exactly one per step, before the others)."""
        g = p.grad
        if g is None:
            return
        if not (0 <= lo < hi <= p.numel()):
            raise ValueError(f"FusedAdam.step_range: [{lo}, {hi}) outside the parameter's {p.numel()} elements")
        if p.dtype != torch.float32 or g.dtype != torch.float32 or not p.is_cuda:
            raise TypeError("FusedAdam: fp32 CUDA parameters and gradients only")
        if not (p.is_contiguous() and g.is_contiguous()):
            raise ValueError("FusedAdam: parameters and gradients must be contiguous")
        group = next(gr for gr in self.param_groups if any(q is p for q in gr["params"]))
        b1, b2 = group["betas"]
        st = self.state[p]
        if len(st) == 0:
            st["step"] = 0
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
        if first:
            st["step"] += 1
        t = st["step"]
        step_size = group["lr"] / (1.0 - b1 ** t)
        bc2_sqrt = (1.0 - b2 ** t) ** 0.5
        o = 4 * lo
        desc = _lib.GstexAdamTensor(p.data_ptr() + o, g.data_ptr() + o, st["exp_avg"].data_ptr() + o,
                                    st["exp_avg_sq"].data_ptr() + o, hi - lo, step_size, bc2_sqrt)
        self._launch({(b1, b2, group["eps"], p.device): [desc]}, zero_grad, 0, grad_scale, skip_flag)

    def _launch(self, batches, zero_grad, grid, grad_scale, skip_flag=None):
        for (b1, b2, eps, dev), items in batches.items():
            st = _lib.stream_of(dev)
            for i in range(0, len(items), _lib.ADAM_MAX_TENSORS):
                chunk = items[i:i + _lib.ADAM_MAX_TENSORS]
                arr = (_lib.GstexAdamTensor * len(chunk))(*chunk)
                flags = (_lib.ADAM_ZERO_GRAD if zero_grad else 0) | ((int(grid) & 0xFFFF) << _lib.ADAM_GRID_SHIFT)
                if skip_flag is not None:
                    _lib.call("gstex_adam_step_guarded", len(chunk), arr, float(b1), float(b2), float(eps), flags,
                              float(grad_scale), _lib.ptr(skip_flag), st)
                elif grad_scale != 1.0:
                    _lib.call("gstex_adam_step_scaled", len(chunk), arr, float(b1), float(b2), float(eps), flags,
                              float(grad_scale), st)
                elif flags:
                    _lib.call("gstex_adam_step_ex", len(chunk), arr, float(b1), float(b2), float(eps), flags, st)
                else:
                    _lib.call("gstex_adam_step", len(chunk), arr, float(b1), float(b2), float(eps), st)
