"""GStexTrainer + FusedAdam + GradSync on the GPU (world size 1 over RCCL): the synced step -- flat gradient
buffer, the raster backward accumulating the texel gradient straight into its slice, the tail collective
started from the backward -- must train exactly like the un-synced step, across an in-place rechart.
(World size > 1 is covered on CPU by tests/test_dist.py; the driver runs the 8-GPU bench.)"""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _assert_trains_alike(name, a, b, what):
    """Parameters of two trainers after the same steps.  Gradients are float-atomic sums (texels always, splat sums
    outside the deterministic mode) whose order varies run to run, and Adam's m / sqrt(v) (eps 1e-15) turns the noise
    of a near-zero gradient into up to one step of update: every element within one step's learning rate, and the
    mean difference within 1e-6 of the largest magnitude (a wrong exchange or update moves the mean far more)."""
    from gstex_amd.model import LRS

    a, b = a.detach().double(), b.detach().double()
    scale = max(float(a.abs().max()), 1e-30)
    d = (a - b).abs()
    err, mean = float(d.max()) / scale, float(d.mean()) / scale
    assert float(d.max()) <= LRS[name] and mean < 1e-6, f"{name}: {what} differs (max {err:.2e}, mean {mean:.2e})"


def test_synced_step_matches_unsynced_across_rechart():
    from gstex_amd.dist import GradSync
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    dev = torch.device("cuda", 0)
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1)
    try:
        sc = make_scene(4000, 80_000, seed=3)
        views = [sphere_view(i, 96, 96).to(dev) for i in range(3)]
        g = torch.Generator().manual_seed(0)
        gts = [torch.rand((96, 96, 3), generator=g).to(dev) for _ in range(3)]
        plain = GStexTrainer(sc, dev, start_step=3000)
        synced = GStexTrainer(sc, dev, start_step=3000)
        sync = GradSync(synced, 1)
        for step in range(5):
            plain.zero_grad()
            plain.forward_backward(views[step % 3], gts[step % 3])
            plain.optimizer_step()
            sync.zero()
            synced.forward_backward(views[step % 3], gts[step % 3])
            assert synced.texture_grad_sink is not None and synced.texture_dc.grad.data_ptr() == \
                sync.flat[sync._tail_off:].data_ptr()
            if step % 2 == 0:
                sync.all_reduce()
                synced.optimizer_step()
            else:  # the exchange inside the step: texel group first, head after its collective (RCCL, world 1)
                synced.optimizer_step(sync=sync)
            if step in (1, 2):
                # step 1: charts for 90 % of the store's rows (fit: the Parameter and the flat buffer are kept);
                # step 2: 130 % (the store grows: a new Parameter, a new buffer and sink at the next zero())
                store, flat = synced.texture_dc, sync.flat
                for tr in (plain, synced):
                    tr.pixel_num = (0.9 if step == 1 else 1.3) * store.shape[0]
                    tr.recharge()
                if step == 1:
                    assert synced.texture_dc is store and synced.n_texels <= store.shape[0]
                else:
                    assert synced.texture_dc is not store and synced.texture_dc.shape[0] > store.shape[0]
                sync.zero()
                assert (sync.flat is flat) == (step == 1), "flat buffer kept in place / rebuilt after growth"
        assert synced.texture_dc.shape == plain.texture_dc.shape
        for (name, a), b in zip(plain.param_groups().items(), synced.param_groups().values()):
            _assert_trains_alike(name, a[0], b[0], "synced step")
    finally:
        dist.destroy_process_group()


def test_deferred_texture_update_across_rechart_and_eval():
    """defer_texture: the texel Adam update of step k run inside step k+1's render (its gradient buffer zeroed by the
    next raster forward); alone and with GradSync's flat buffer (world 1), across an in-place rechart and an eval
    render, it must train like the plain step."""
    from gstex_amd.dist import GradSync
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    dev = torch.device("cuda", 0)
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1)
    try:
        sc = make_scene(4000, 80_000, seed=5)
        views = [sphere_view(i, 96, 96).to(dev) for i in range(3)]
        g = torch.Generator().manual_seed(1)
        gts = [torch.rand((96, 96, 3), generator=g).to(dev) for _ in range(3)]
        plain = GStexTrainer(sc, dev, start_step=3000)
        alone = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
        synced = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
        assert alone.defer_texture and synced.defer_texture
        sync = GradSync(synced, 1)
        for step in range(5):
            for tr in (plain, alone):
                tr.zero_grad()
                tr.forward_backward(views[step % 3], gts[step % 3])
                tr.optimizer_step()
            sync.zero()
            synced.forward_backward(views[step % 3], gts[step % 3])
            sync.all_reduce()
            synced.optimizer_step()
            if step == 1:
                for tr in (plain, alone, synced):
                    tr.recharge()
            if step == 2:
                ev = [tr.eval_render(views[0])["rgb"] for tr in (plain, alone)]
                assert float((ev[0] - ev[1]).abs().max()) < 1e-4
        for tr in (alone, synced):
            tr.wait_texture()
        torch.cuda.synchronize()
        # the persistent texel-gradient buffers hold the last gradient until the next differentiable raster forward
        # zeroes them (gstex_raster_fwd_zero), before its backward accumulates into them; a fused-render trainer keeps
        # it in the second buffer of its pair (the current one was zeroed by the last raster backward)
        last = alone._tex_grad_next if alone._tex_grad_next is not None else alone.texture_dc.grad
        assert float(last.abs().max()) > 0.0
        for tr in (alone, synced):
            tr.render(views[0])
        torch.cuda.synchronize()
        assert float(alone.texture_dc.grad.abs().max()) == 0.0
        assert float(sync.flat[sync._tail_off:].abs().max()) == 0.0
        for other in (alone, synced):
            for (name, a), b in zip(plain.param_groups().items(), other.param_groups().values()):
                _assert_trains_alike(name, a[0], b[0], "deferred texel update")
    finally:
        dist.destroy_process_group()


def test_deferred_texture_update_matches_plain_step():
    """defer_texture: step k's texel Adam update runs inside step k+1's render (while the host reads back the pair
    count); alone and under GradSync (world 1, the overlapped exchange of optimizer_step(sync=...)), across an
    in-place and a growing rechart and an eval render, it must train like the plain step."""
    from gstex_amd.dist import GradSync
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    dev = torch.device("cuda", 0)
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1)
    try:
        sc = make_scene(4000, 80_000, seed=6)
        views = [sphere_view(i, 96, 96).to(dev) for i in range(3)]
        g = torch.Generator().manual_seed(2)
        gts = [torch.rand((96, 96, 3), generator=g).to(dev) for _ in range(3)]
        plain = GStexTrainer(sc, dev, start_step=3000)
        alone = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
        synced = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
        assert alone.defer_texture and synced.defer_texture
        sync = GradSync(synced, 1)
        for step in range(6):
            for tr in (plain, alone):
                tr.zero_grad()
                tr.forward_backward(views[step % 3], gts[step % 3])
                tr.optimizer_step()
            sync.zero()
            synced.forward_backward(views[step % 3], gts[step % 3])
            synced.optimizer_step(sync=sync)
            assert alone._pending_tex is not None and synced._pending_tex is not None
            if step in (1, 3):
                for tr in (plain, alone, synced):
                    tr.pixel_num = (0.9 if step == 1 else 1.3) * tr.texture_dc.shape[0]
                    tr.recharge()
            if step == 2:
                ev = [tr.eval_render(views[0])["rgb"] for tr in (plain, alone)]
                assert float((ev[0] - ev[1]).abs().max()) < 1e-4
        for tr in (alone, synced):
            tr.wait_texture()
        torch.cuda.synchronize()
        # the persistent texel-gradient buffers hold the last gradient until the next differentiable raster forward
        # zeroes them (gstex_raster_fwd_zero); a fused-render trainer keeps it in the second buffer of its pair (the
        # current one was zeroed by the last raster backward, gstex_raster_bwd_zero)
        last = alone._tex_grad_next if alone._tex_grad_next is not None else alone.texture_dc.grad
        assert float(last.abs().max()) > 0.0
        for tr in (alone, synced):
            tr.render(views[0])
        torch.cuda.synchronize()
        assert float(alone.texture_dc.grad.abs().max()) == 0.0
        assert float(sync.flat[sync._tail_off:].abs().max()) == 0.0
        for other in (alone, synced):
            assert other.texture_dc.shape == plain.texture_dc.shape
            for (name, a), b in zip(plain.param_groups().items(), other.param_groups().values()):
                _assert_trains_alike(name, a[0], b[0], "deferred texel update")
    finally:
        dist.destroy_process_group()


def test_skipped_step_leaves_no_stale_texel_gradient():
    """a backward whose optimizer step is skipped (e.g. a non-finite loss) must not leak its texel
    gradient into the next step.  zero_grad() (alone) and GradSync.zero() (data-parallel, world 1 over RCCL) mark the
    persistent sink for re-zeroing by the next raster forward: zero_grad, backward, no step, zero_grad, backward, step
    must train like the plain trainer doing only the second backward and step."""
    from gstex_amd.dist import GradSync
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    dev = torch.device("cuda", 0)
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1)
    try:
        sc = make_scene(3000, 60_000, seed=13)
        views = [sphere_view(i, 96, 96).to(dev) for i in range(2)]
        g = torch.Generator().manual_seed(6)
        gts = [torch.rand((96, 96, 3), generator=g).to(dev) for _ in range(2)]
        plain = GStexTrainer(sc, dev, start_step=3000)
        deferred = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
        synced = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
        sync = GradSync(synced, 1)
        for step in range(3):
            plain.zero_grad()
            plain.forward_backward(views[1], gts[1])
            plain.optimizer_step()
            deferred.zero_grad()
            deferred.forward_backward(views[0], gts[0])  # its step is skipped
            deferred.zero_grad()
            deferred.forward_backward(views[1], gts[1])
            deferred.optimizer_step()
            sync.zero()
            synced.forward_backward(views[0], gts[0])  # skipped
            sync.zero()
            synced.forward_backward(views[1], gts[1])
            synced.optimizer_step(sync=sync)
        for tr in (deferred, synced):
            tr.wait_texture()
        torch.cuda.synchronize()
        for other in (deferred, synced):
            for (name, a), b in zip(plain.param_groups().items(), other.param_groups().values()):
                _assert_trains_alike(name, a[0], b[0], "skipped step")
    finally:
        dist.destroy_process_group()


def test_texture_sink_accumulates_the_renders_of_one_step():
    """Two views per optimizer step (gradient accumulation): the persistent texel-gradient sink of a deferred-update
    trainer is zeroed by the step's first raster forward only, so both views' texel gradients reach the update -- it
    must train like the plain trainer, whose autograd accumulates them."""
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    dev = torch.device("cuda", 0)
    sc = make_scene(3000, 60_000, seed=12)
    views = [sphere_view(i, 96, 96).to(dev) for i in range(2)]
    g = torch.Generator().manual_seed(5)
    gts = [torch.rand((96, 96, 3), generator=g).to(dev) for _ in range(2)]
    plain = GStexTrainer(sc, dev, start_step=3000)
    deferred = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
    for _ in range(3):
        for tr in (plain, deferred):
            tr.zero_grad()
            tr.forward_backward(views[0], gts[0])
            tr.forward_backward(views[1], gts[1])
            tr.optimizer_step()
    deferred.wait_texture()
    torch.cuda.synchronize()
    for (name, a), b in zip(plain.param_groups().items(), deferred.param_groups().values()):
        _assert_trains_alike(name, a[0], b[0], "texel sink over two renders")


def test_pair_capacity_step_trains_like_the_readback_step():
    """Capacity mode (ops.PairCapacity, the default): pair buffers sized from a capacity, the pair total kept on the
    device -- must train like the reference's read-back sizing (pair_capacity=False), deferred texel update included,
    across a growing rechart; and a step of it performs no host synchronisation (no .item() / .cpu() / pinned copy /
    stream, event or device synchronisation; the pair totals are read later with non-blocking event queries)."""
    from gstex_amd import ops
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    dev = torch.device("cuda", 0)
    sc = make_scene(4000, 80_000, seed=21)
    views = [sphere_view(i, 96, 96).to(dev) for i in range(3)]
    g = torch.Generator().manual_seed(8)
    gts = [torch.rand((96, 96, 3), generator=g).to(dev) for _ in range(3)]
    sync = GStexTrainer(sc, dev, start_step=3000, defer_texture=True, pair_capacity=False)
    capd = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
    assert sync.pairs is None and capd.pairs is not None
    for step in range(5):
        for tr in (sync, capd):
            tr.zero_grad()
            tr.forward_backward(views[step % 3], gts[step % 3])
            tr.optimizer_step()
        if step == 1:
            for tr in (sync, capd):
                tr.pixel_num = 1.3 * tr.texture_dc.shape[0]
                tr.recharge()
    # a step in capacity mode, with every host-synchronising call counted
    calls = []

    def spy(name, fn):
        def w(*a, **k):
            calls.append(name)
            return fn(*a, **k)
        return w

    saved = {}
    patch = [(torch.Tensor, n) for n in ("item", "cpu", "tolist", "numpy", "__bool__", "__float__", "__int__")]
    patch += [(torch.cuda, "synchronize"), (torch.cuda.Stream, "synchronize"), (torch.cuda.Event, "synchronize"),
              (ops, "_start_count"), (ops, "_finish_count")]
    for obj, n in patch:
        saved[(obj, n)] = getattr(obj, n)
        setattr(obj, n, spy(n, saved[(obj, n)]))
    try:
        capd.zero_grad()
        capd.forward_backward(views[0], gts[0])
        capd.optimizer_step()
    finally:
        for (obj, n), fn in saved.items():
            setattr(obj, n, fn)
    assert calls == [], f"host synchronisation inside a capacity-mode step: {calls}"
    sync.zero_grad()
    sync.forward_backward(views[0], gts[0])
    sync.optimizer_step()
    for tr in (sync, capd):
        tr.wait_texture()
    torch.cuda.synchronize()
    capd._poll_pairs()
    assert capd.skipped_steps == [] and capd.pairs.max_total > 0
    assert capd.pairs.capacity >= capd.pairs.max_total
    for (name, a), b in zip(sync.param_groups().items(), capd.param_groups().values()):
        _assert_trains_alike(name, a[0], b[0], "capacity-mode step")


@pytest.mark.parametrize("det", [False, True])
def test_pair_capacity_overflow_skips_the_update_and_grows(request, det):
    """A capacity below the pair total: the render comes out empty, every Adam launch of the step (the deferred texel
    update included) leaves parameters and moments untouched, the host finds the overflow from the totals it polls,
    grows the capacity, and the next step trains.  det: under torch.use_deterministic_algorithms(True) (per-pair rows
    sized by the capacity, ADVICE r04: setup_bwd must not address rows past them when the total overflows)."""
    if det:
        request.getfixturevalue("deterministic")
    from gstex_amd import ops
    from gstex_amd.loss import photometric_loss
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    dev = torch.device("cuda", 0)
    sc = make_scene(3000, 60_000, seed=22)
    view = sphere_view(0, 96, 96).to(dev)
    gt = torch.rand((96, 96, 3), generator=torch.Generator().manual_seed(9)).to(dev)
    tr = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
    tr.pairs = ops.PairCapacity(dev, capacity=1000)  # far below this scene's ~20k pairs
    before = [p.detach().clone() for p in tr.parameters()]
    # one step whose single render overflows (a second render inside the step would race the host's poll: a poll
    # between the renders grows the capacity, and the later render's total then fits -- the step is still skipped,
    # because the renders of a step OR their flags, but the renders' outputs would differ)
    tr.zero_grad()
    out = tr.render(view)
    assert float(out["alpha"].abs().max()) == 0.0  # every tile empty
    loss, _ = photometric_loss(out["img"], out["tex"], out["alpha"], tr.background, gt)
    loss.backward()
    tr.optimizer_step()
    tr.wait_texture()
    torch.cuda.synchronize()
    for p, q in zip(before, tr.parameters()):
        assert torch.equal(p, q.detach()), "an overflowed step changed a parameter"
    for st in tr.optimizer.state.values():
        assert float(st["exp_avg"].abs().max()) == 0.0 and float(st["exp_avg_sq"].abs().max()) == 0.0
    with pytest.warns(UserWarning, match="exceeded the pair capacity"):
        tr._poll_pairs()
    assert tr.skipped_steps == [3000] and tr.pairs.capacity > tr.pairs.max_total > 1000
    tr.zero_grad()
    tr.forward_backward(view, gt)
    tr.optimizer_step()
    tr.wait_texture()
    torch.cuda.synchronize()
    tr._poll_pairs()
    assert tr.skipped_steps == [3000]
    assert any(not torch.equal(p, q.detach()) for p, q in zip(before, tr.parameters()))


def test_fused_overflow_does_not_skip_later_steps():
    """the fused training render's pair guard must reset the step's flag at its first render even when the
    double-buffered texel gradient needs no zeroing (the previous backward zeroed it).  A fused step that overflows
    is skipped; the eight fused steps after it -- including step s + 8, which reuses its step_control slot -- update."""
    from gstex_amd import ops
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    dev = torch.device("cuda", 0)
    sc = make_scene(3000, 60_000, seed=23)
    view = sphere_view(0, 96, 96).to(dev)
    gt = torch.rand((96, 96, 3), generator=torch.Generator().manual_seed(10)).to(dev)
    tr = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
    tr.pairs = ops.PairCapacity(dev, capacity=1000)  # far below this scene's ~20k pairs
    assert tr._fused_ok(False, None) and tr._double_buffered()

    def step():
        tr.zero_grad()
        tr.forward_backward(view, gt)
        tr.optimizer_step()
        tr.wait_texture()
        torch.cuda.synchronize()

    before = [p.detach().clone() for p in tr.parameters()]
    step()  # step 3000: overflows on the fused path
    for p, q in zip(before, tr.parameters()):
        assert torch.equal(p, q.detach()), "an overflowed fused step changed a parameter"
    with pytest.warns(UserWarning, match="exceeded the pair capacity"):
        tr._poll_pairs()
    assert tr.skipped_steps == [3000]
    for k in range(1, 10):  # steps 3001 .. 3009; 3008 uses the overflowed step's flag slot
        prev = [p.detach().clone() for p in tr.parameters()]
        step()
        assert float(tr.step_control[(tr.step - 1) % 8]) == 0.0, f"step {tr.step - 1}'s guard flag left set"
        assert all(not torch.equal(p, q.detach()) for p, q in zip(prev, tr.parameters())
                   if q.grad is not None), f"fused step {tr.step - 1} was skipped"
    tr._poll_pairs()
    assert tr.skipped_steps == [3000]


def test_two_renders_per_step_under_overlapped_gradsync():
    """gradient accumulation over two views per step with the default overlapped exchange (a trainer that
    does not defer its texel update, the tail's collective started from the first raster backward): the second render
    accumulates into GradSync's side buffer, reduced and added once the tail has landed -- trains like the plain
    trainer (world 1 over RCCL)."""
    from gstex_amd.dist import GradSync
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    dev = torch.device("cuda", 0)
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1)
    try:
        sc = make_scene(3000, 60_000, seed=14)
        views = [sphere_view(i, 96, 96).to(dev) for i in range(2)]
        g = torch.Generator().manual_seed(7)
        gts = [torch.rand((96, 96, 3), generator=g).to(dev) for _ in range(2)]
        plain = GStexTrainer(sc, dev, start_step=3000)
        synced = GStexTrainer(sc, dev, start_step=3000)
        sync = GradSync(synced, 1)
        assert not sync.head_first
        for step in range(3):
            plain.zero_grad()
            plain.forward_backward(views[0], gts[0])
            plain.forward_backward(views[1], gts[1])
            plain.optimizer_step()
            sync.zero()
            synced.forward_backward(views[0], gts[0])
            assert sync._work is not None  # the tail's collective started from the first raster backward
            synced.forward_backward(views[1], gts[1])
            synced.optimizer_step(sync=sync)
        torch.cuda.synchronize()
        for (name, a), b in zip(plain.param_groups().items(), synced.param_groups().values()):
            _assert_trains_alike(name, a[0], b[0], "two renders per step under GradSync")
    finally:
        dist.destroy_process_group()
