"""Fused multi-tensor Adam (``gstex_adam_step``) for the GStex parameter groups.

Drop-in for the reference's ``torch.optim.Adam(params, lr, eps=1e-15)`` per group
(gstex_configs.py:207-244, engine/optimizers.py:158-171): the same update, the same
per-parameter ``state`` ({"step", "exp_avg", "exp_avg_sq"}) and ``param_groups``, so code that resets a
parameter's moments (the rechart, gstex.py:799-826) keeps working.  All parameters of all groups are
updated by one HIP launch (16 tensors per launch) instead of torch's ~7 foreach passes.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


class AdamSchedule:
    """Per-step Adam bias corrections on the device, for training steps captured into hipGraphs
    (gstex_adam_step_scheduled, gstex_amd.graphs.StepGraphs).

    A captured launch cannot take a new step_size / bias_correction2_sqrt each replay, so for every parameter this keeps
    a device table of those two fp32 scalars for steps t0, t0 + 1, ... -- the same python-double expressions
    FusedAdam.step evaluates per call, rounded to fp32 the same way -- and the captured update reads row
    (t_capture - t0) + counter, where `counter` (a device int32) is advanced by one at the end of every replayed step.
    Replay r therefore applies the corrections of step t_capture + r, exactly what the eager step r would.  shift(n)
    slides every table n steps forward and takes n off the counter (stream-ordered) before the rows run out."""

    def __init__(self, optimizer, device, rows: int = 8192):
        self.rows = int(rows)
        self.device = torch.device(device)
        self.counter = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._t0, self._tables, self._groups = {}, {}, {}
        self.updates = {}  # id(param) -> updates registered since reset_updates() (one per parameter per step)
        for group in optimizer.param_groups:
            for p in group["params"]:
                t0 = int(optimizer.state[p].get("step", 0)) + 1 if p in optimizer.state else 1
                self._t0[id(p)] = t0
                self._groups[id(p)] = group
                self._tables[id(p)] = torch.from_numpy(self._host_table(group, t0)).to(self.device)

    def _host_table(self, group, t0: int) -> np.ndarray:
        b1, b2 = group["betas"]
        lr = group["lr"]
        out = np.empty((self.rows, 2), dtype=np.float32)
        for r in range(self.rows):
            t = t0 + r
            out[r, 0] = lr / (1.0 - b1 ** t)  # FusedAdam.step's step_size and bc2_sqrt, fp32-rounded like c_float
            out[r, 1] = (1.0 - b2 ** t) ** 0.5
        return out

    def entry(self, p, t: int):
        """(table pointer, row of counter = 0) for parameter p's update at step t."""
        key = id(p)
        if key not in self._tables:
            raise RuntimeError("AdamSchedule: a parameter added after the schedule was built (re-capture the step)")
        self.updates[key] = self.updates.get(key, 0) + 1
        return self._tables[key].data_ptr(), t - self._t0[key]

    def reset_updates(self):
        self.updates = {}

    def shift(self, n: int):
        """Slide every table n steps forward and take n off the device counter (stream-ordered, between replays)."""
        for key, tab in self._tables.items():
            self._t0[key] += n
            tab.copy_(torch.from_numpy(self._host_table(self._groups[key], self._t0[key])))
        self.counter.sub_(n)


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        if lr < 0 or eps < 0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid Adam hyper-parameters lr={lr} betas={betas} eps={eps}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps))
        # an AdamSchedule while a training step is being captured into a hipGraph (gstex_amd.graphs): the launches then
        # read their bias corrections from its device tables (gstex_adam_step_scheduled)
        self.schedule = None

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
                sched = self.schedule.entry(p, t) if self.schedule is not None else None
                batches.setdefault(key, []).append((desc, sched))
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
        if self.schedule is not None:
            raise RuntimeError("FusedAdam.step_range: not supported inside a captured step (StepGraphs is single-GPU)")
        self._launch({(b1, b2, group["eps"], p.device): [(desc, None)]}, zero_grad, 0, grad_scale, skip_flag)

    def _launch(self, batches, zero_grad, grid, grad_scale, skip_flag=None):
        for (b1, b2, eps, dev), items in batches.items():
            st = _lib.stream_of(dev)
            for i in range(0, len(items), _lib.ADAM_MAX_TENSORS):
                chunk = items[i:i + _lib.ADAM_MAX_TENSORS]
                arr = (_lib.GstexAdamTensor * len(chunk))(*[d for d, _ in chunk])
                flags = (_lib.ADAM_ZERO_GRAD if zero_grad else 0) | ((int(grid) & 0xFFFF) << _lib.ADAM_GRID_SHIFT)
                if chunk[0][1] is not None:  # captured step: bias corrections from the AdamSchedule's tables
                    sch = _lib.GstexAdamSchedule()
                    sch.counter = self.schedule.counter.data_ptr()
                    for j, (_, (tab, base)) in enumerate(chunk):
                        sch.table[j], sch.base[j], sch.rows[j] = tab, base, self.schedule.rows
                    _lib.call("gstex_adam_step_scheduled", len(chunk), arr, float(b1), float(b2), float(eps), flags,
                              float(grad_scale), _lib.ptr(skip_flag), ctypes.byref(sch), st)
                elif skip_flag is not None:
                    _lib.call("gstex_adam_step_guarded", len(chunk), arr, float(b1), float(b2), float(eps), flags,
                              float(grad_scale), _lib.ptr(skip_flag), st)
                elif grad_scale != 1.0:
                    _lib.call("gstex_adam_step_scaled", len(chunk), arr, float(b1), float(b2), float(eps), flags,
                              float(grad_scale), st)
                elif flags:
                    _lib.call("gstex_adam_step_ex", len(chunk), arr, float(b1), float(b2), float(eps), flags, st)
                else:
                    _lib.call("gstex_adam_step", len(chunk), arr, float(b1), float(b2), float(eps), st)
