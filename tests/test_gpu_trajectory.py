"""Training-trajectory parity proxy for north_star's "PSNR within 0.05 dB of reference on Blender/chair" (VERDICT r04
next #4).  The Blender data is absent (parity of the PSNR clause itself stays unpinned), so the proxy compares two
trainers on the same synthetic task:
  * the HIP path: gstex_amd.model.GStexTrainer as bench.py runs it (fused activations / SH / loss / Adam, the deferred
    texel update, capacity-sized pair buffers, float-atomic gradient sums);
  * an oracle-driven trainer (tests/oracle_trainer.py): the CPU oracle's fp32 forward and torch autograd backward,
    eager loss, torch.optim.Adam -- the same views, learning rates, rechart schedule and seed.
Both start from the same random-init scene (3,000 splats, 45,000 texels) and fit the images a different seeded scene
renders (the oracle, 64 x 64, eight sphere poses), one pose per step for 150 steps from step 0, so the SH degree ramp
min(step // interval, 3) (gstex.py:1103, sh_degree_interval 1000 in the reference, 20 here) runs through degrees
0, 1, 2 and 3, with recharts after steps 60 and 120 (build_chart_every, gstex.py:202, 890-895; 100 in the
reference).  (Sized to run in about 100 s on the GPU box: the oracle trainer's CPU time dominates.)  Every 10 steps both render a held-out pose and the PSNR is taken as the reference's metric does (torchmetrics PeakSignalNoiseRatio(data_range=1.0) on the composited rgb,
gstex.py:350, 1262-1272): 10 log10(1 / MSE).  Pass: |PSNR_hip - PSNR_oracle| <= 0.05 dB at every logged step, and the
task must actually train (PSNR up by >= 1 dB).  The per-group parameter drift between the two trainers is printed.
Measured (profiles/r06_trajectory.log, 4,000 splats / 200 steps): |dPSNR| <= 0.0031 dB over the 21 logged steps,
10.25 -> 21.03 dB, 181 s; at this size (profiles/r06_trajectory_3k.log) |dPSNR| <= 0.0005 dB, 10.74 -> 20.60 dB, 124 s.
"""
import math
import time

import pytest
import torch

from gstex_amd.scene import make_scene, sphere_view
from oracle import raster as O
from oracle_trainer import OracleTrainer

pytestmark = pytest.mark.gpu

N, T, HW, STEPS, EVERY, RECHARTS, POSES, SH_EVERY = 3000, 45000, 64, 150, 10, (60, 120), 8, 20


def psnr(rgb, gt):
    mse = float(((rgb.double() - gt.double()) ** 2).mean())
    return 10.0 * math.log10(1.0 / mse)


def teacher_images(views):
    """The target images: a different seeded scene rendered by the oracle (white background, as the trainers')."""
    sc = make_scene(N, T, seed=99, opacity=0.6)
    means, scales, quats, opac = sc.activated()
    uv0, umap, vmap = sc.uv_mapping()
    g = torch.Generator().manual_seed(98)
    rgbs = torch.rand((N, 3), generator=g)
    out = []
    for v in views:
        cam = O.Camera(v.viewmat, v.fx, v.fy, v.cx, v.cy, v.H, v.W, 16, v.c2w[:3, 3])
        centers, extents = O.aabb_2d(means, scales, 1.0, quats, cam)
        _, depths = O.project_points(means, cam)
        inp = O.RasterInputs(sc.texture_dims, centers, extents, depths, rgbs, opac, means, scales, 1.0, quats, uv0,
                             umap, vmap, sc.texture, cam, (1 << 9) | (1 << 10), None)
        o32, _, _ = O.rasterize(inp, grad_dtype=torch.float32)
        out.append(torch.clamp(o32["img"] + o32["tex"][:, :, :3] + (1 - o32["alpha"][:, :, None]), 0, 1).detach())
    return out


@pytest.mark.timeout(900)
def test_training_trajectory_psnr_matches_the_oracle_trainer():
    from gstex_amd.model import GStexTrainer

    torch.set_num_threads(min(16, torch.get_num_threads()))
    dev = torch.device("cuda", 0)
    views = [sphere_view(i, HW, HW, n_views=POSES + 1) for i in range(POSES + 1)]
    gts = teacher_images(views)
    train_views, eval_view, eval_gt = views[:POSES], views[POSES], gts[POSES]
    scene = make_scene(N, T, seed=5)
    hip = GStexTrainer(scene, dev, start_step=0, sh_degree_interval=SH_EVERY, defer_texture=True)
    ref = OracleTrainer(scene, start_step=0, sh_degree_interval=SH_EVERY)
    dviews = [v.to(dev) for v in views]
    dgts = [g.to(dev) for g in gts]
    log = []
    t0 = time.time()

    def measure(step):
        with torch.no_grad():
            p_hip = psnr(hip.render(dviews[POSES], sh_degree_now=hip.sh_degree_now())["rgb"].cpu(), eval_gt)
            p_ref = psnr(ref.render(eval_view), eval_gt)
        log.append((step, p_hip, p_ref))
        print(f"step {step:3d}: PSNR hip {p_hip:.4f} dB, oracle {p_ref:.4f} dB, diff {p_hip - p_ref:+.4f} dB "
              f"({time.time() - t0:.0f} s)", flush=True)

    measure(0)
    for step in range(STEPS):
        k = step % POSES
        hip.zero_grad()
        hip.forward_backward(dviews[k], dgts[k])
        hip.optimizer_step()
        ref.zero_grad()
        ref.forward_backward(train_views[k], gts[k])
        ref.optimizer_step()
        if step + 1 in RECHARTS:
            hip.recharge()
            ref.recharge()
            # each trainer charts its own scales (build_charts is deterministic): after 100 steps of float-atomic
            # noise a few splats sit on the other side of a ceil() and get another texel count, which the PSNR absorbs
            dh = hip.texture_dims.cpu()
            n_diff = int((dh[:, :2] != ref.texture_dims[:, :2]).any(-1).sum())
            print(f"rechart after step {step + 1}: {n_diff} of {N} splats charted differently; texels "
                  f"{int(dh[:, 0].long().mul(dh[:, 1].long()).sum())} (hip) vs "
                  f"{int(ref.texture_dims[:, 0].long().mul(ref.texture_dims[:, 1].long()).sum())} (oracle)")
            assert n_diff <= N // 50, "the recharts diverged"
        if (step + 1) % EVERY == 0:
            measure(step + 1)
        if (step + 1) % SH_EVERY == 0 and step + 1 <= 3 * SH_EVERY:
            assert hip.sh_degree_now() == ref.sh_degree_now() == (step + 1) // SH_EVERY
    hip.wait_texture()
    torch.cuda.synchronize()
    dh, dr = hip.texture_dims.cpu().long(), ref.texture_dims.long()
    same = (dh[:, :2] == dr[:, :2]).all(-1)  # splats charted alike by both recharts: their texel blocks correspond
    for name, ph, pr in zip(hip.param_groups(), hip.parameters(), ref.parameters()):
        a, b = ph.detach().cpu().double(), pr.detach().double()
        if name == "texture_dc":  # per splat block (the stores' offsets differ after a splat charted differently)
            idx_h = torch.cat([torch.arange(int(dh[i, 2]), int(dh[i, 2] + dh[i, 0] * dh[i, 1])) for i in range(N) if same[i]])
            idx_r = torch.cat([torch.arange(int(dr[i, 2]), int(dr[i, 2] + dr[i, 0] * dr[i, 1])) for i in range(N) if same[i]])
            a, b = a[idx_h], b[idx_r]
        n = min(a.shape[0], b.shape[0])
        d = (a[:n] - b[:n]).abs()
        print(f"  {name:14s} drift max {float(d.max()):.3e}, mean {float(d.mean()):.3e} "
              f"(max |param| {float(b.abs().max()):.3e})")
    assert hip.skipped_steps == []
    assert log[-1][2] - log[0][2] >= 1.0, "the task did not train: the proxy would say nothing"
    worst = max(abs(h - r) for _, h, r in log)
    assert worst <= 0.05, f"PSNR of the HIP trainer differs from the oracle trainer's by {worst:.4f} dB"
