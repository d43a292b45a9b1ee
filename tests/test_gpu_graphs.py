"""hipGraph-captured training steps (gstex_amd.graphs.StepGraphs, bench.py's N = 1 step) against the eager step.

Under torch.use_deterministic_algorithms(True) the splat gradients are bitwise reproducible (per-pair rows summed in a
fixed order); the texel gradients stay float-atomic sums (order varies run to run), so the texel group trains with
lr = 0 here: its values then stay fixed and every other group's gradient is reproducible.  A trainer whose steps are
graph replays must then hold exactly the parameters, Adam moments and step counts of an eager trainer after the same
steps -- the device-side bias-correction tables (gstex_adam_step_scheduled) included, across two table shifts
(rows = 16), eager steps between replays (the graphs are re-captured) and a final deferred texel update; the texel
moments agree within the float-atomic noise."""
import os

import pytest
import torch

# Opt-in (GSTEX_GRAPH_TESTS=1): a capture pattern this module no longer uses (a slot captured into a shared pool after
# other slots of that pool had been replayed) faulted the GPU in round 5, and the back-to-back capture policy that
# replaced it has not run on the GPU since; the product paths (bench.py's default, smoke(), every other test) never
# capture a graph.
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(os.environ.get("GSTEX_GRAPH_TESTS", "0") != "1",
                                 reason="hipGraph step tests run only with GSTEX_GRAPH_TESTS=1 (see module comment)")]


def _pair(n_poses=3, hw=128):
    from gstex_amd.model import GStexTrainer
    from gstex_amd.scene import make_scene, sphere_view

    dev = torch.device("cuda", 0)
    sc = make_scene(12_000, 200_000, seed=11)
    views = [sphere_view(i, hw, hw, n_views=n_poses).to(dev) for i in range(n_poses)]
    g = torch.Generator().manual_seed(5)
    gts = [torch.rand((hw, hw, 3), generator=g).to(dev) for _ in range(n_poses)]
    a = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
    b = GStexTrainer(sc, dev, start_step=3000, defer_texture=True)
    for tr in (a, b):
        for g in tr.optimizer.param_groups:
            if g["name"] == "texture_dc":
                g["lr"] = 0.0  # (see the module docstring)
    return a, b, views, gts


def _body(tr, views, gts):
    def body(k):
        tr.zero_grad()
        tr.forward_backward(views[k], gts[k])
        tr.optimizer_step()
    return body


def _assert_same(a, b):
    a.wait_texture()
    b.wait_texture()
    torch.cuda.synchronize()
    assert a.step == b.step
    for (name, pa), pb in zip(a.param_groups().items(), b.parameters()):
        pa = pa[0]
        assert torch.equal(pa, pb), f"{name}: parameters differ (max {float((pa - pb).abs().max()):.3e})"
        sa, sb = a.optimizer.state.get(pa, {}), b.optimizer.state.get(pb, {})
        assert sa.keys() == sb.keys(), name
        if not sa:  # never updated (no gradient: features_dc)
            continue
        assert sa["step"] == sb["step"], f"{name}: Adam step {sa['step']} vs {sb['step']}"
        if name == "texture_dc":  # float-atomic gradients: the moments agree within their noise
            for key in ("exp_avg", "exp_avg_sq"):
                d = float((sa[key] - sb[key]).abs().max())
                assert d <= 1e-3 * max(float(sa[key].abs().max()), 1e-30), f"{name} {key}: {d:.3e}"
            continue
        assert torch.equal(sa["exp_avg"], sb["exp_avg"]) and torch.equal(sa["exp_avg_sq"], sb["exp_avg_sq"]), name


@pytest.mark.timeout(300)
def test_graph_replays_match_eager_steps_bitwise():
    from gstex_amd.graphs import StepGraphs

    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        a, b, views, gts = _pair()
        ea, eb = _body(a, views, gts), _body(b, views, gts)
        graphs = StepGraphs(b, eb, len(views), rows=16)
        for s in range(2):  # eager steps size the pair capacity
            ea(s % 3)
            eb(s % 3)
        graphs.capture()  # every slot, back to back
        for s in range(2, 26):  # 24 replays: the 16-row tables shift twice (before replays 15 and 23)
            ea(s % 3)
            graphs.replay(s % 3)
        assert graphs.replays == 24 and graphs._row0 == 16 and not b.skipped_steps
        _assert_same(a, b)
        for s in range(26, 29):  # eager steps between replays: the next replay re-captures (all slots, back to back)
            ea(s % 3)
            eb(s % 3)
        for s in range(29, 33):
            ea(s % 3)
            graphs.replay(s % 3)
        assert graphs.replays == 4 and graphs.captured == 3
        _assert_same(a, b)
        graphs.close()
    finally:
        torch.use_deterministic_algorithms(False)


@pytest.mark.timeout(300)
def test_graph_kernel_timing_events():
    """The raster backward timed inside the graphs: one fresh event pair per replay, durations close to the eager
    launches' (the same kernel), and nothing recorded while timing is off."""
    from gstex_amd import ops
    from gstex_amd.graphs import StepGraphs

    a, b, views, gts = _pair()
    eb = _body(b, views, gts)
    graphs = StepGraphs(b, eb, len(views), timed={"gstex_raster_bwd"})
    eb(0)
    eb(1)
    graphs.capture()  # every slot, back to back (never a capture between replays of the same pool)
    ops.set_kernel_timing(True, names={"gstex_raster_bwd"})
    for s in range(4):
        eb(s % 3)
    eager = ops.kernel_times()["gstex_raster_bwd"]
    graphs.capture()  # (after those eager steps: re-captured here rather than at the first replay)
    ops.set_kernel_timing(True, names={"gstex_raster_bwd"})
    for s in range(6):
        graphs.replay(s % 3)
    replayed = ops.kernel_times()["gstex_raster_bwd"]
    ops.set_kernel_timing(False)
    for s in range(3):
        graphs.replay(s % 3)
    torch.cuda.synchronize()
    assert len(replayed) == 6 and all(t > 0 for t in replayed), replayed
    med_e, med_r = sorted(eager)[len(eager) // 2], sorted(replayed)[3]
    print(f"raster bwd: eager {eager} ms, replayed {replayed} ms")
    assert 0.5 * med_e < med_r < 2.0 * med_e
    graphs.close()
