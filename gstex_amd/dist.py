"""Data-parallel gradient exchange for multi-view GStex training (one process per GPU).

Replaces the reference's DDP wrapper (pipelines/base_pipeline.py:281-283, 25 MB buckets,
find_unused_parameters=True) with ONE flat fp32 gradient buffer per rank:

* every parameter's .grad is a view into the buffer, so backward accumulates straight into it
  (no bucket copies) and one RCCL all-reduce (torch "nccl" backend = RCCL on ROCm, over xGMI)
  averages it — ~165 MB at 200k splats / 1e7 texels, a single large message that RCCL spreads
  over all xGMI links;
* the buffer is rebuilt whenever a parameter changes size (the texel store after a rechart,
  gstex.py:890-895, models/jagged_texture.py:53-64) — the case where the reference's DDP buckets
  go stale.

Parameters that receive no gradient in a step (features_dc under SH colour) are reduced as zeros,
matching DDP's find_unused_parameters semantics.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib


class GradSync:
    """overlap_tail: the last parameter (the texel store, ~73 % of the bytes at cfg3) gets its own asynchronous
    all-reduce as soon as its gradient is final, overlapping the collective with the rest of the backward
    (setup_bwd, SH, activations); all_reduce() then reduces the head of the buffer and waits for both.

    A trainer that exposes ``texture_grad_sink`` / ``texture_grad_ready`` (gstex_amd.model.GStexTrainer) gets
    the tail slice of the flat buffer as the raster backward's texel-gradient target: the kernel accumulates
    straight into the buffer (no separate zero-filled gradient tensor, no autograd accumulation pass) and the
    tail collective starts right after that kernel is enqueued.  Other parameter holders use a
    post-accumulate-grad hook on the tail parameter.

    The buffer layout is keyed on parameter identity and shape: a rechart that reuses the texel store in place
    (GStexTrainer.recharge while the new charts fit its capacity) keeps the buffer; one that replaces the
    Parameter rebuilds it.  One backward per all_reduce(): gradient accumulation over several backward passes
    is not supported (the tail would be reduced after the first).

    Several differentiable renders per step (gradient accumulation over views) with the tail started early: the
    trainer asks texture_grad_route(first) for each render's texel-gradient target; once the tail's collective is on
    the wire, later renders of the step accumulate into a side buffer instead, which the step reduces and adds to the
    slice after the tail has landed."""

    def __init__(self, trainer, world_size: int, group=None, overlap_tail: bool = True, tail_chunks: int = 4):
        self.trainer = trainer
        self.world = world_size
        self.group = group
        self.overlap_tail = overlap_tail
        # head first: the tail's collective in this many pieces, so that a chunked texel update (all_reduce_and_step
        # step_tail_range) steps each piece while the next one is still on the wire
        self.tail_chunks = max(1, int(tail_chunks))
        self._key = None
        self.flat = None
        self._tail_off = 0
        self._hook = None
        self._hooked = None
        self._work = None
        self._extra = None  # the side buffer of renders after the tail's early start (texture_grad_route)
        self._extra_live = False
        self._sink = hasattr(trainer, "texture_grad_sink")
        # head first (a trainer that defers its texel update into the next step, GStexTrainer defer_texture): the
        # tail's collective is not started from the raster backward but queued right behind the head's at the step,
        # so the head (45 MB) lands first, the next step starts on it, and the tail (120 MB) only has to land by that
        # step's raster forward
        self.head_first = bool(getattr(trainer, "defer_texture", False))
        # a trainer with a pair-capacity guard (GStexTrainer.step_control): its per-step overflow flags live in the
        # first CTRL elements of the flat buffer, so the head collective sums them over the ranks and every rank's
        # Adam launches skip the same steps
        self._ctrl = hasattr(trainer, "step_control")
        # phase timing (bench.py at N > 1): when a dict, HIP events recorded on the compute stream as the head's
        # ("head") and the whole tail's ("tail") collectives land -- with the raster kernels' own events they give
        # the exposed exchange time per step
        self.phase_events = None
        self.rebuild()

    def _params(self):
        return self.trainer.parameters()

    ALIGN = 64  # elements
    CTRL = 64  # elements in front of the parameters: the trainer's step_control ring (pair-capacity guard flags)

    @staticmethod
    def _layout(params):
        return [(id(p), tuple(p.shape)) for p in params]

    def rebuild(self):
        params = self._params()
        key = self._layout(params)
        if key == self._key and self.flat is not None:
            return False
        if self.flat is not None and hasattr(self.trainer, "wait_texture"):
            self.trainer.wait_texture()  # a side-stream texel update may still read the old buffer
        # every slice starts on a 256-B boundary (the fused Adam's float4 path needs 16-B aligned gradients)
        offs = []
        total = self.CTRL if self._ctrl else 0
        for p in params:
            offs.append(total)
            total += -(-p.numel() // self.ALIGN) * self.ALIGN
        dev = params[0].device
        self.flat = torch.zeros(total, device=dev, dtype=torch.float32)
        if self._ctrl:  # the flags of steps still in flight move with the buffer
            ring = self.trainer.step_control
            self.flat[:ring.numel()].copy_(ring)
            self.trainer.step_control = self.flat[:ring.numel()]
        self._z0 = self.CTRL if self._ctrl else 0  # zero() leaves the control block alone
        self._offs = offs
        for p, off in zip(params, offs):
            p.grad = self.flat[off:off + p.numel()].view_as(p)
        self._key = key
        self._tail_off = offs[-1]
        if self._sink:
            self.trainer.texture_grad_sink = params[-1].grad
            self.trainer.texture_grad_ready = (self._tail_ready_sink if self.overlap_tail and not self.head_first
                                               else None)
            self.trainer.texture_grad_route = self._route
            # the trainer's second (double-buffered) texel-gradient buffer is never used once the flat buffer's slice
            # is the sink (GStexTrainer._double_buffered() is False): free it
            if getattr(self.trainer, "_tex_grad_next", None) is not None:
                self.trainer._tex_grad_next = None
                self.trainer._next_zeroed = False
        else:
            self._install_hook(params[-1])
        return True

    def _install_hook(self, tail):
        if not self.overlap_tail or self._hooked is tail:
            return
        if self._hook is not None:
            self._hook.remove()
        self._hooked = tail
        self._hook = tail.register_post_accumulate_grad_hook(self._tail_ready)

    def _start_tail(self):
        self._work = dist.all_reduce(self.flat[self._tail_off:], op=dist.ReduceOp.SUM, group=self.group,
                                     async_op=True)

    def _tail_ready_sink(self):
        # the raster backward has just been enqueued on the compute stream: the collective is stream-ordered
        # after it and overlaps the rest of the backward.  A second backward before all_reduce() would add into the
        # slice the in-flight collective is reading: refused (one backward per all_reduce(), class docstring)
        if self._work is not None:
            raise RuntimeError("GradSync: a second backward before all_reduce() (its texel gradient would race the "
                               "collective still reading the flat buffer)")
        self._start_tail()

    def _route(self, first: bool):
        """(target, zero, ready) of one render's texel gradient: the flat buffer's slice (zeroed by that render when
        `first`, the tail collective started once its backward is enqueued), or -- when an earlier render of the step
        already started the tail's collective -- the side buffer, reduced and added by the step."""
        tail = self.trainer.texture_grad_sink
        if self._work is None:
            return tail, first, self.trainer.texture_grad_ready
        if self._extra is None or self._extra.shape != tail.shape:
            self._extra = torch.zeros_like(tail)
            self._extra_live = True
            return self._extra, False, None
        zero = not self._extra_live
        self._extra_live = True
        return self._extra, zero, None

    def _fold_extra(self):
        """After the tail's collective has landed: reduce the side buffer of the step's later renders into it."""
        if self._extra_live:
            dist.all_reduce(self._extra, op=dist.ReduceOp.SUM, group=self.group)
            self.flat[self._tail_off:self._tail_off + self._extra.numel()].add_(self._extra.view(-1))
            self._extra_live = False

    def _tail_ready(self, param):
        # fires once the texel gradient is final for this backward; the view is still the flat buffer's
        if self._work is None and param.grad is not None and param.grad.data_ptr() == self.flat[self._tail_off:].data_ptr():
            self._start_tail()

    @property
    def nbytes(self) -> int:
        return self.flat.numel() * 4

    def zero(self):
        if self._work is not None:
            raise RuntimeError("GradSync.zero(): the previous backward's all_reduce() was never called")
        reset = getattr(self.trainer, "reset_texture_grad", None)
        if reset is not None:
            reset()  # the sink (the texel slice) is zeroed by the next differentiable raster forward
        if self.rebuild():
            return  # a new buffer is zero
        if getattr(self.trainer, "texture_grad_zeroed_by_update", False):
            # the texel slice is zeroed by the next differentiable raster forward (gstex_raster_fwd_zero); filling it
            # here would pre-empt the deferred texel update (defer_texture) still reading it
            self.flat[self._z0:self._tail_off].zero_()
        else:
            self.flat[self._z0:].zero_()

    def all_reduce(self):
        """Average the flat gradient buffer over all ranks (the tail's collective may already be running).

        Every .grad must still be its view of the buffer: a zero_grad(set_to_none=True) after zero() (trainer or
        optimizer) lets autograd write fresh tensors, which are folded back into the buffer here (a parameter whose
        .grad is None took no gradient; the texel store's slice keeps what the raster backward wrote into it)."""
        work, self._work = self._work, None
        params = self._params()
        if self._layout(params) != self._key:
            if work is not None:
                work.wait()
                raise RuntimeError("GradSync.all_reduce(): the parameters changed between backward and all_reduce() "
                                   "(call zero() after a rechart, before the backward)")
            self.rebuild_if_detached()
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
        else:
            # the tail is the texel store: with a running collective its slice is final (written by the kernel)
            self._reattach(params, skip_tail=work is not None)
            if work is not None:
                dist.all_reduce(self.flat[:self._tail_off], op=dist.ReduceOp.SUM, group=self.group)
                work.wait()
                self._fold_extra()
            else:
                dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
        self.flat.mul_(1.0 / self.world)

    def tail_bounds(self, n: int):
        """The head-first tail collective's pieces: [lo, hi) element ranges of the tail parameter, 1024-element
        (4 KiB) aligned, at most tail_chunks of them."""
        k = max(1, min(self.tail_chunks, n // 1024))
        step = -(-(-(-n // k)) // 1024) * 1024
        return [(lo, min(n, lo + step)) for lo in range(0, n, step)]

    def all_reduce_and_step(self, step_tail, step_head, defer_tail: bool = False, step_tail_range=None):
        """A data-parallel optimizer step with the collectives overlapped (the trainer's optimizer_step(sync=...)).

        The tail collective (the texel store, started from the raster backward) is followed on the wire by the head's;
        step_tail(scale) runs as soon as the tail is reduced, so the texel group's update (73 % of the parameters)
        overlaps the head collective, then step_head(scale) after it.  Both get scale = 1 / world to apply to the
        SUMMED gradients (FusedAdam grad_scale: the same fp32 product as averaging first, without the separate pass
        over the buffer), so after this call the buffer holds sums, not averages.  Without a running tail collective
        (overlap_tail=False, or no backward hook fired) this is all_reduce() followed by both steps at scale 1.
        defer_tail: the head is stepped now and the tail's step is returned as a callable instead of run (the trainer's
        defer_texture: it runs inside the next step's render, after the tail collective has had that much longer).
        step_tail_range(scale, lo, hi, first) (head first only): the tail's update of its elements [lo, hi), so the
        tail's collective goes out in pieces (tail_bounds) and each piece is stepped as soon as it lands; `first` marks
        the piece that advances the optimizer's step count."""
        work, self._work = self._work, None
        params = self._params()
        if defer_tail and self.head_first and work is None and self._layout(params) == self._key:
            self._reattach(params, skip_tail=self._sink)
            head = dist.all_reduce(self.flat[:self._tail_off], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            bounds = self.tail_bounds(params[-1].numel()) if step_tail_range is not None else [(0, params[-1].numel())]
            tails = [dist.all_reduce(self.flat[self._tail_off + lo:self._tail_off + hi], op=dist.ReduceOp.SUM,
                                     group=self.group, async_op=True) for lo, hi in bounds]
            scale = 1.0 / self.world
            head.wait()
            self._mark("head")
            step_head(scale)

            def tail_step():
                if step_tail_range is None:
                    tails[0].wait()
                    self._mark("tail")
                    step_tail(scale)
                    return
                # each piece stepped as soon as it has landed, while the next ones are still on the wire
                for i, ((lo, hi), w) in enumerate(zip(bounds, tails)):
                    w.wait()
                    if i == len(tails) - 1:
                        self._mark("tail")
                    step_tail_range(scale, lo, hi, i == 0)
            return tail_step
        if work is None or self._layout(params) != self._key:
            if work is not None:
                work.wait()
                raise RuntimeError("GradSync.all_reduce_and_step(): the parameters changed between backward and the "
                                   "step (call zero() after a rechart, before the backward)")
            self.all_reduce()
            step_head(1.0)
            if defer_tail:
                return lambda: step_tail(1.0)
            step_tail(1.0)
            return None
        self._reattach(params, skip_tail=True)
        head = dist.all_reduce(self.flat[:self._tail_off], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        scale = 1.0 / self.world
        if self._ctrl and not defer_tail:
            # the step's guard flag is agreed only once the head (which carries it) has landed
            work.wait()
            self._fold_extra()
            self._mark("tail")
            head.wait()
            self._mark("head")
            step_tail(scale)
            step_head(scale)
            return None
        if defer_tail:
            head.wait()
            self._mark("head")
            step_head(scale)

            def tail():
                work.wait()
                self._fold_extra()
                self._mark("tail")
                step_tail(scale)
            return tail
        work.wait()
        self._fold_extra()
        self._mark("tail")
        step_tail(scale)
        head.wait()
        self._mark("head")
        step_head(scale)
        return None

    def _mark(self, phase):
        """A timing event on the current stream (phase_events enabled): the point a collective has landed at."""
        if self.phase_events is not None:
            ev = _lib.TimingEvent()  # fence-free (timing only), comparable with the raster launches' events
            ev.record()
            self.phase_events.setdefault(phase, []).append(ev)

    def _reattach(self, params, skip_tail=False):
        """Point every .grad back at its slice of `flat`, copying a detached gradient in (None: zero, except the
        texel store's slice when the raster backward accumulated straight into it -- the sink)."""
        last = len(params) - 1
        for i, (p, off) in enumerate(zip(params, self._offs)):
            view = self.flat[off:off + p.numel()]
            if p.grad is not None and p.grad.data_ptr() == view.data_ptr():
                continue
            g = p.grad
            p.grad = view.view_as(p)
            if i == last and (skip_tail or self._sink):
                if g is not None and g.data_ptr() != view.data_ptr():
                    p.grad.add_(g)  # an autograd gradient on top of the sink's accumulation (none in GStexTrainer)
                continue
            if g is not None:
                p.grad.copy_(g)
            else:
                p.grad.zero_()

    def rebuild_if_detached(self):
        # autograd may have replaced a .grad that was not a view of `flat` (e.g. first step after
        # a parameter was re-created): fold it back into the buffer before reducing.
        params = self._params()
        if self._layout(params) != self._key:
            grads = [p.grad.detach().clone() if p.grad is not None else None for p in params]
            self._key = None
            self.rebuild()
            for p, g in zip(params, grads):
                if g is not None:
                    p.grad.copy_(g)
            return
        for p, off in zip(params, self._offs):
            view = self.flat[off:off + p.numel()]
            if p.grad is None or p.grad.data_ptr() != view.data_ptr():
                g = p.grad
                p.grad = view.view_as(p)
                if g is not None:
                    p.grad.copy_(g)
                else:
                    p.grad.zero_()
