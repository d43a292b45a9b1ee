"""Multi-view data parallelism (one process per device): the flat-buffer gradient all-reduce of
gstex_amd.dist.GradSync, exercised with world_size 2 on the gloo backend (CPU)."""
import os
import socket
from types import SimpleNamespace

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gstex_amd.dist import GradSync


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Params:
    def __init__(self, rank, n_tex):
        g = torch.Generator().manual_seed(7)
        self.means = torch.nn.Parameter(torch.randn(10, 3, generator=g))
        self.unused = torch.nn.Parameter(torch.randn(4, 3, generator=g))  # like features_dc: no grad
        self.texture = torch.nn.Parameter(torch.randn(n_tex, 3, generator=g))

    def parameters(self):
        return [self.means, self.unused, self.texture]


def _worker(rank, world, port, q, overlap=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = _Params(rank, 6)
        sync = GradSync(p, world, overlap_tail=overlap)
        sync.zero()
        # rank-dependent "loss": gradients differ per rank (independent cameras)
        ((rank + 1) * p.means.sum() + (rank + 2) * (p.texture ** 2).sum()).backward()
        assert p.means.grad.data_ptr() == sync.flat.data_ptr(), "grads must be views of the flat buffer"
        assert (sync._work is not None) == overlap, "the texel-gradient collective starts inside backward"
        sync.all_reduce()
        exp_means = torch.full((10, 3), (1 + 2) / 2.0)
        exp_tex = 2 * p.texture.detach() * ((2 + 3) / 2.0)
        ok1 = torch.allclose(p.means.grad, exp_means) and torch.allclose(p.texture.grad, exp_tex)
        ok1 = ok1 and torch.all(p.unused.grad == 0)
        # rechart: the texel store changes size -> the buffer is rebuilt and still reduces correctly
        p.texture = torch.nn.Parameter(torch.ones(9, 3))
        sync.zero()
        ((rank + 1) * p.texture.sum()).backward()
        sync.all_reduce()
        # (slices start on GradSync.ALIGN-element boundaries: 30, 12 and 27 elements -> offsets 0, 64, 128)
        ok2 = torch.allclose(p.texture.grad, torch.full((9, 3), 1.5)) and sync._offs == [0, 64, 128]
        ok2 = ok2 and sync.flat.numel() == 128 + 64
        q.put((rank, bool(ok1), bool(ok2)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [True, False])
def test_grad_all_reduce_world2(overlap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, overlap)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in procs]
    for pr in procs:
        pr.join(timeout=60)
    assert sorted(r[0] for r in res) == [0, 1]
    assert all(r[1] for r in res), "flat all-reduce did not average the gradients"
    assert all(r[2] for r in res), "flat buffer not rebuilt after the texel store changed size"


class _SinkTrainer:
    """The parameter layout of gstex_amd.model.GStexTrainer (7 groups, texel store last) and its texel-gradient
    sink protocol, on CPU: `backward()` plays the raster backward (accumulates into the sink and calls the ready
    callback) plus autograd for the other parameters."""

    def __init__(self, n=12, n_tex=40):
        g = torch.Generator().manual_seed(3)
        P = lambda *s: torch.nn.Parameter(torch.randn(*s, generator=g))  # noqa: E731
        self.means, self.features_dc, self.features_rest = P(n, 3), P(n, 3), P(n, 15, 3)
        self.opacities, self.scales, self.quats = P(n, 1), P(n, 3), P(n, 4)
        self.texture_dc = P(n_tex, 3)
        self.texture_grad_sink = None
        self.texture_grad_ready = None
        self.texture_grad_route = None
        self._fresh = True

    def parameters(self):
        return [self.means, self.features_dc, self.features_rest, self.opacities, self.scales, self.quats,
                self.texture_dc]

    def zero_grad(self, set_to_none=True):  # torch.optim.Optimizer.zero_grad semantics (GStexTrainer.zero_grad)
        for p in self.parameters():
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    def backward(self, rank, scale=1.0):
        w = float(rank + 1) * scale
        loss = w * (self.means.sum() + self.features_rest.sum() + 2 * self.opacities.sum() + self.scales.sum()
                    + self.quats.sum())
        loss.backward()  # features_dc unused under SH colour, like the real step
        assert self.texture_grad_sink is not None, "GradSync must hand the texel slice to the raster backward"
        if self.texture_grad_route is not None and scale != 1.0:
            # several renders in one step (GStexTrainer.render): the per-render target, zeroed by its first render
            sink, zero, ready = self.texture_grad_route(self._fresh)
            self._fresh = False
            if zero:
                sink.zero_()
        else:
            sink, ready = self.texture_grad_sink, self.texture_grad_ready
        sink.add_(w * self.texture_dc.detach())  # the kernel's accumulation
        if ready is not None:
            ready()


def _trainer_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = _SinkTrainer()
        sync = GradSync(tr, world)
        res = {}
        mean_w = sum(r + 1 for r in range(world)) / world
        for step in range(3):
            sync.zero()
            tr.backward(rank)
            res[f"tail_started_{step}"] = sync._work is not None
            sync.all_reduce()
            ok = torch.allclose(tr.texture_dc.grad, mean_w * tr.texture_dc.detach())
            ok = ok and torch.allclose(tr.means.grad, torch.full_like(tr.means, mean_w))
            ok = ok and torch.allclose(tr.opacities.grad, torch.full_like(tr.opacities, 2 * mean_w))
            ok = ok and bool(torch.all(tr.features_dc.grad == 0))
            res[f"ok_{step}"] = bool(ok)
            flat_before = sync.flat.data_ptr()
            if step == 0:  # rechart that fits the store: same Parameter, written in place -> no rebuild
                with torch.no_grad():
                    tr.texture_dc.data[:30] = 1.0
            elif step == 1:  # rechart that grows the store: a new Parameter -> rebuilt buffer and sink
                tr.texture_dc = torch.nn.Parameter(torch.ones(55, 3))
            sync.zero()
            res[f"rebuilt_{step}"] = sync.flat.data_ptr() != flat_before
            tr.backward(rank)
            sync.all_reduce()
            res[f"after_rechart_{step}"] = bool(torch.allclose(tr.texture_dc.grad, mean_w * tr.texture_dc.detach()))
        # zero_grad(set_to_none=True) after zero(): autograd writes detached .grad tensors and the
        # kernel still fills the sink; all_reduce() must fold them back and reduce everything exactly once
        for step in range(2):
            sync.zero()
            tr.zero_grad()
            tr.backward(rank)
            detached = tr.means.grad.data_ptr() != sync.flat.data_ptr()
            sync.all_reduce()
            ok = detached and torch.allclose(tr.texture_dc.grad, mean_w * tr.texture_dc.detach())
            ok = ok and torch.allclose(tr.means.grad, torch.full_like(tr.means, mean_w))
            ok = ok and torch.allclose(tr.quats.grad, torch.full_like(tr.quats, mean_w))
            ok = ok and bool(torch.all(tr.features_dc.grad == 0))
            ok = ok and tr.means.grad.data_ptr() == sync.flat.data_ptr()  # re-attached to the buffer
            res[f"set_to_none_{step}"] = bool(ok)
        # the overlapped exchange inside the optimizer step (GStexTrainer.optimizer_step(sync=...)): the texel step
        # runs once the tail collective has landed, the head step after the head collective; both see SUMS and the
        # scale 1 / world
        sync.zero()
        tr.backward(rank)
        calls = []
        sync.all_reduce_and_step(lambda sc: calls.append(("tail", sc, tr.texture_dc.grad.clone())),
                                 lambda sc: calls.append(("head", sc, tr.means.grad.clone(), tr.features_dc.grad.clone())))
        sum_w = mean_w * world
        res["overlap_order"] = [c[0] for c in calls] == ["tail", "head"]
        res["overlap_scale"] = all(abs(c[1] - 1.0 / world) < 1e-15 for c in calls)
        res["overlap_sums"] = bool(torch.allclose(calls[0][2], sum_w * tr.texture_dc.detach())
                                   and torch.allclose(calls[1][2], torch.full_like(tr.means, sum_w))
                                   and torch.all(calls[1][3] == 0))
        # deferred tail (GStexTrainer defer_texture): the head is stepped at once, the tail's step comes back as a
        # callable, run later (in the next step's render) with the same sums and scale
        sync.zero()
        tr.backward(rank)
        calls = []
        pending = sync.all_reduce_and_step(lambda sc: calls.append(("tail", sc, tr.texture_dc.grad.clone())),
                                           lambda sc: calls.append(("head", sc, tr.means.grad.clone())),
                                           defer_tail=True)
        res["defer_head_first"] = [c[0] for c in calls] == ["head"] and callable(pending)
        pending()
        res["defer_tail_later"] = ([c[0] for c in calls] == ["head", "tail"]
                                   and all(abs(c[1] - 1.0 / world) < 1e-15 for c in calls)
                                   and bool(torch.allclose(calls[1][2], sum_w * tr.texture_dc.detach())))
        # a second backward without all_reduce() in between is refused: by zero(), and by the sink's ready callback
        # (its kernel would add into the slice the running collective reads)
        sync.zero()
        tr.backward(rank)
        try:
            sync.zero()
            res["double_backward_refused"] = False
        except RuntimeError:
            res["double_backward_refused"] = True
        try:
            tr.backward(rank)
            res["double_backward_sink_refused"] = False
        except RuntimeError:
            res["double_backward_sink_refused"] = True
        sync.all_reduce()
        # head first (a trainer that defers its texel update, GStexTrainer defer_texture): the backward starts no
        # collective; the step queues the head's then the tail's, steps the head, and returns the tail's step
        tr2 = _SinkTrainer()
        tr2.defer_texture = True
        sync2 = GradSync(tr2, world)
        sync2.zero()
        tr2.backward(rank)
        res["head_first_no_early_tail"] = sync2.head_first and sync2._work is None
        calls = []
        pending = sync2.all_reduce_and_step(lambda sc: calls.append(("tail", sc, tr2.texture_dc.grad.clone())),
                                            lambda sc: calls.append(("head", sc, tr2.means.grad.clone())),
                                            defer_tail=True)
        first = [c[0] for c in calls] == ["head"]
        pending()
        res["head_first_sums"] = (first and [c[0] for c in calls] == ["head", "tail"]
                                  and all(abs(c[1] - 1.0 / world) < 1e-15 for c in calls)
                                  and bool(torch.allclose(calls[0][2], torch.full_like(tr2.means, sum_w)))
                                  and bool(torch.allclose(calls[1][2], sum_w * tr2.texture_dc.detach())))
        # head first with a chunked texel update (GStexTrainer passes step_tail_range): the tail's collective goes out
        # in tail_bounds pieces, each stepped once it has landed; together they cover the tail once, in order, the
        # first one flagged
        tr3 = _SinkTrainer(n_tex=1500)
        tr3.defer_texture = True
        sync3 = GradSync(tr3, world)
        sync3.zero()
        tr3.backward(rank)
        calls = []
        pending = sync3.all_reduce_and_step(
            lambda sc: calls.append(("tail", sc)),
            lambda sc: calls.append(("head", sc, tr3.means.grad.clone())), defer_tail=True,
            step_tail_range=lambda sc, lo, hi, first: calls.append(
                ("range", sc, lo, hi, first, tr3.texture_dc.grad.view(-1)[lo:hi].clone())))
        pending()
        rng = [c for c in calls if c[0] == "range"]
        whole = (sum_w * tr3.texture_dc.detach()).view(-1)
        res["chunked_tail"] = (len(rng) > 1 and [c[0] for c in calls] == ["head"] + ["range"] * len(rng)
                               and rng[0][2] == 0 and rng[-1][3] == whole.numel()
                               and all(a[3] == b[2] for a, b in zip(rng, rng[1:]))
                               and [c[4] for c in rng] == [True] + [False] * (len(rng) - 1)
                               and all(abs(c[1] - 1.0 / world) < 1e-15 for c in rng)
                               and all(bool(torch.allclose(c[5], whole[c[2]:c[3]])) for c in rng)
                               and all(sync3._offs[i] % GradSync.ALIGN == 0 for i in range(len(sync3._offs))))
        # several renders in one step with the tail started early by the first one's backward: the later
        # renders accumulate into GradSync's side buffer, reduced and added once the tail has landed
        tr4 = _SinkTrainer()
        sync4 = GradSync(tr4, world)
        for step in range(2):
            sync4.zero()
            tr4._fresh = True
            tr4.backward(rank, scale=1.0 + 1e-9)  # (scale != 1: through texture_grad_route)
            started = sync4._work is not None
            tr4.backward(rank, scale=2.0)
            tr4.backward(rank, scale=3.0)
            if step == 0:
                sync4.all_reduce()
                got = tr4.texture_dc.grad.clone()
            else:
                calls = []
                sync4.all_reduce_and_step(lambda sc: calls.append(sc * tr4.texture_dc.grad.clone()),
                                          lambda sc: calls.append(sc * tr4.means.grad.clone()))
                got = calls[0]
            want = (1.0 + 1e-9 + 2.0 + 3.0) * mean_w * tr4.texture_dc.detach()
            res[f"multi_render_{step}"] = started and bool(torch.allclose(got, want, rtol=1e-6))
        # the pair-capacity guard's control block (a trainer with step_control): the first CTRL elements of the flat
        # buffer, summed over the ranks by the head's collective, left alone by zero(), carried over a rebuild
        tr5 = _SinkTrainer()
        tr5.step_control = torch.zeros(8)
        sync5 = GradSync(tr5, world)
        ok = sync5._offs[0] == GradSync.CTRL and tr5.step_control.data_ptr() == sync5.flat.data_ptr()
        sync5.zero()
        tr5.step_control[3] = 1.0 if rank == 0 else 0.0  # rank 0's render of step 3 overflowed
        tr5.backward(rank)
        sync5.all_reduce_and_step(lambda sc: None, lambda sc: None)
        ok = ok and float(tr5.step_control[3]) > 0 and float(tr5.step_control.abs().sum()) == float(tr5.step_control[3])
        sync5.zero()
        ok = ok and float(tr5.step_control[3]) > 0  # zero() keeps the flags of steps in flight
        tr5.texture_dc = torch.nn.Parameter(torch.ones(55, 3))
        sync5.zero()  # rebuild: a new buffer, the flags copied over
        ok = ok and float(tr5.step_control[3]) > 0 and tr5.step_control.data_ptr() == sync5.flat.data_ptr()
        res["ctrl_block"] = bool(ok)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_trainer_layout_sink_and_recharts_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in procs]
    for pr in procs:
        pr.join(timeout=60)
    for rank, r in res:
        for step in range(3):
            assert r[f"tail_started_{step}"], "the texel collective must start from the raster backward"
            assert r[f"ok_{step}"], f"rank {rank} step {step}: wrong averaged gradients"
            assert r[f"after_rechart_{step}"], f"rank {rank} step {step}: wrong gradients after a rechart"
        assert not r["rebuilt_0"], "an in-place rechart must keep the flat buffer"
        assert r["rebuilt_1"], "a grown texel store must rebuild the flat buffer"
        assert r["double_backward_refused"]
        assert r["double_backward_sink_refused"]
        assert r["overlap_order"] and r["overlap_scale"] and r["overlap_sums"], r
        assert r["defer_head_first"] and r["defer_tail_later"], r
        assert r["head_first_no_early_tail"] and r["head_first_sums"], r
        assert r["chunked_tail"], r
        assert r["multi_render_0"] and r["multi_render_1"], r
        assert r["ctrl_block"], r
        for step in range(2):
            assert r[f"set_to_none_{step}"], f"rank {rank}: zero_grad(set_to_none) after zero() mis-reduced (step {step})"
