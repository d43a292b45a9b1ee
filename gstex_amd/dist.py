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


class GradSync:
    def __init__(self, trainer, world_size: int, group=None):
        self.trainer = trainer
        self.world = world_size
        self.group = group
        self._shapes = None
        self.flat = None
        self.rebuild()

    def _params(self):
        return self.trainer.parameters()

    def rebuild(self):
        params = self._params()
        shapes = [tuple(p.shape) for p in params]
        if shapes == self._shapes and self.flat is not None:
            return False
        total = sum(p.numel() for p in params)
        dev = params[0].device
        self.flat = torch.zeros(total, device=dev, dtype=torch.float32)
        off = 0
        for p in params:
            n = p.numel()
            p.grad = self.flat[off:off + n].view_as(p)
            off += n
        self._shapes = shapes
        return True

    @property
    def nbytes(self) -> int:
        return self.flat.numel() * 4

    def zero(self):
        self.rebuild()
        self.flat.zero_()

    def all_reduce(self):
        """Average the flat gradient buffer over all ranks (one collective)."""
        self.rebuild_if_detached()
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
        self.flat.mul_(1.0 / self.world)

    def rebuild_if_detached(self):
        # autograd may have replaced a .grad that was not a view of `flat` (e.g. first step after
        # a parameter was re-created): fold it back into the buffer before reducing.
        params = self._params()
        if [tuple(p.shape) for p in params] != self._shapes:
            grads = [p.grad.detach().clone() if p.grad is not None else None for p in params]
            self._shapes = None
            self.rebuild()
            for p, g in zip(params, grads):
                if g is not None:
                    p.grad.copy_(g)
            return
        off = 0
        for p in params:
            n = p.numel()
            view = self.flat[off:off + n]
            if p.grad is None or p.grad.data_ptr() != view.data_ptr():
                g = p.grad
                p.grad = view.view_as(p)
                if g is not None:
                    p.grad.copy_(g)
                else:
                    p.grad.zero_()
            off += n
