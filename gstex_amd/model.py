"""GStex train-step harness around the HIP rasterizer.

Reproduces the parts of the reference's GStexModel that sit either side of the hot path, so the
"train-step ms" metric is measured on the same work the reference does per step:
  * parameter activations            gstex.py:1059-1066
  * UV frames (detached)             gstex.py:975-990
  * preprocessing                    gstex.py:1077-1080   (project_points / get_aabb_2d / tiles)
  * SH colour with the DC zeroed     gstex.py:1099-1114
  * texture = SH2RGB(texture_dc)     gstex.py:1093-1094,1119
  * texture_gaussians                gstex.py:1133-1162
  * background composite             gstex.py:1204-1205
  * loss 0.8 L1 + 0.2 (1 - SSIM)     gstex.py:1301-1322 (pytorch_msssim SSIM semantics; fused HIP
                                     kernels in gstex_amd.loss, eager torch path kept for reference)
  * per-group Adam, eps 1e-15        gstex_configs.py:207-244, engine/optimizers.py:158-171
                                     (one fused HIP launch, gstex_amd.optim.FusedAdam)
The rechart every 100 steps (gstex.py:890-914) is provided by `recharge()`.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from . import ops
from .activations import activate, sh_rest
from .loss import depth_to_normal, gaussian_window, geometry_loss, photometric_loss, scheduled
from .optim import FusedAdam
from .charts import SH2RGB, build_charts, get_uv_mapping, texture_dims_to_query
from .scene import Scene, View

# gstex-blender-nvs optimizer settings (gstex_configs.py:207-244)
LRS = {
    "xyz": 5 * 1.6e-5,
    "features_dc": 0.0025,
    "features_rest": 0.0025 / 20,
    "opacity": 0.05,
    "scaling": 0.005,
    "rotation": 0.001,
    "texture_dc": 1e-3,
}
DEFAULT_SETTINGS = (1 << 9) | (1 << 10)
SH_C0 = 0.28209479177387814  # SH2RGB(x) = SH_C0 * x + 0.5 (gstex.py:94-99)


def _gauss_window(size=11, sigma=1.5, device=None):
    return gaussian_window(size, sigma).to(device)  # the same fp32 weights the fused kernels use


_BANDS: dict = {}


def _band(n: int, win: torch.Tensor) -> torch.Tensor:
    """(n, n-k+1) banded matrix M with M[i+j, i] = win[j]: x @ M is the valid 1-D correlation."""
    key = (n, win.numel(), win.device, float(win[0]))
    m = _BANDS.get(key)
    if m is None:
        k = win.numel()
        out = n - k + 1
        m = torch.zeros(n, out, device=win.device, dtype=win.dtype)
        idx = torch.arange(out, device=win.device)
        for j in range(k):
            m[idx + j, idx] = win[j]
        _BANDS[key] = m
    return m


def ssim(x: torch.Tensor, y: torch.Tensor, data_range=1.0, win_size=11, sigma=1.5, K=(0.01, 0.03)) -> torch.Tensor:
    """pytorch_msssim.SSIM(data_range=1, size_average=True, channel=3) on (1,C,H,W): separable
    gaussian window, valid convolution, mean over the map (gstex.py:351,1303).

    The separable valid filter runs as two banded GEMMs (hipBLASLt): MIOpen serves this depthwise
    11-tap convolution with its naive kernels, which cost more than the whole rasterizer."""
    H, W = x.shape[-2:]
    g = _gauss_window(win_size, sigma, x.device)
    bw = _band(W, g)
    bh = _band(H, g)

    def filt(t):  # (..., H, W) -> (..., H-k+1, W-k+1)
        return torch.matmul(bh.t(), torch.matmul(t, bw))

    C1 = (K[0] * data_range) ** 2
    C2 = (K[1] * data_range) ** 2
    maps = filt(torch.stack([x, y, x * x, y * y, x * y], 0))
    mu1, mu2 = maps[0], maps[1]
    s11 = maps[2] - mu1 * mu1
    s22 = maps[3] - mu2 * mu2
    s12 = maps[4] - mu1 * mu2
    cs = (2 * s12 + C2) / (s11 + s22 + C2)
    sm = ((2 * mu1 * mu2 + C1) / (mu1 * mu1 + mu2 * mu2 + C1)) * cs
    return sm.mean()


@dataclass
class StepOutput:
    loss: torch.Tensor
    rgb: torch.Tensor


class GStexTrainer:
    """Holds the GStex parameters on one device and runs forward/backward/Adam steps."""

    def __init__(self, scene: Scene, device, sh_degree: int = 3, settings: int = DEFAULT_SETTINGS,
                 pixel_num: float | None = None, background=(1.0, 1.0, 1.0), fused_adam: bool = True,
                 fused_loss: bool = True, fused_activations: bool = True, geometry_outputs: bool = False,
                 sh_degree_interval: int = 1000, fix_init: bool = False, start_step: int = 0,
                 defer_texture: bool = False, lambda_normal=0.0, lambda_reg=0.0, use_normal_loss: bool = False,
                 pair_capacity: bool | None = None, fused_step: bool | None = None):
        self.device = torch.device(device)
        d = self.device
        P = lambda t: torch.nn.Parameter(t.detach().to(d).contiguous())  # noqa: E731
        # the geometry parameters (what decides which (pixel, splat) pairs exist) share one allocation, each segment
        # 16-B aligned (the fused Adam's float4 path): `geometry_flat` snapshots / restores all four in one copy
        geo = [scene.means, scene.log_scales, scene.quats, scene.opacity_logits]
        sizes = [int(t.numel()) for t in geo]
        self.geometry_flat = torch.zeros(sum((n + 3) // 4 * 4 for n in sizes), device=d, dtype=torch.float32)
        views, off = [], 0
        for t, n in zip(geo, sizes):
            v = self.geometry_flat[off:off + n].view(t.shape)
            v.copy_(t.detach().to(d))
            views.append(torch.nn.Parameter(v))
            off += (n + 3) // 4 * 4
        self.means, self.scales, self.quats, self.opacities = views
        self.features_dc = P(scene.features_dc)
        self.features_rest = P(scene.features_rest)
        # the texel parameter stores the SH-DC value; the raster reads SH2RGB of it (gstex.py:1119).  Like the
        # reference's JaggedTexture (jagged_texture.py:36-64) it is a capacity store: rows [0, n_texels) are the
        # texels of the current charts, the store only grows at a rechart, and the raster takes the whole store
        # (texture_dims never index past n_texels), so its gradient needs no slice-backward copy
        tex_dc = (scene.texture[:, :3] - 0.5) / 0.28209479177387814
        self.texture_dc = P(tex_dc)
        self.n_texels = int(tex_dc.shape[0])
        self.texture_dims = scene.texture_dims.to(d).contiguous()
        self.mappings = scene.mappings.to(d).contiguous()
        self.sh_degree = sh_degree
        self.settings = settings
        self.pixel_num = pixel_num if pixel_num is not None else float(scene.texture.shape[0])
        self.background = torch.tensor(background, dtype=torch.float32, device=d)
        # the raster's own background is zero (the composite adds the real one, gstex.py:1204): one cached tensor
        self._bg_zero = torch.zeros_like(self.background)
        self._one = torch.ones((), dtype=torch.float32, device=d)
        self.step = start_step
        self.sh_degree_interval = sh_degree_interval  # gstex.py:182
        self.fix_init = fix_init  # gstex.py:209 (DTU configs): SH view directions (x, -z, y), gstex.py:1104-1108
        self.fused_adam = fused_adam
        self.fused_loss = fused_loss
        self.fused_activations = fused_activations
        # depth / distortion / normal renders: only for losses or views that read them (the reference's normal
        # and distortion weights default to 0, gstex.py:198-201, so its training loss uses none of them)
        self.geometry_outputs = geometry_outputs
        # the 2DGS regularisers of get_loss_dict (gstex.py:198-201, 207, 1218-1220, 1313-1317): weights as numbers or
        # [before, after, switch_step] schedules; a non-zero weight renders depth / distortion / normal for the step
        self.lambda_normal = lambda_normal
        self.lambda_reg = lambda_reg
        self.use_normal_loss = use_normal_loss
        # set by gstex_amd.dist.GradSync: the flat-buffer slice the raster backward accumulates the texel gradient
        # into, and the callback that starts its collective (None: autograd owns the texel gradient)
        self.texture_grad_sink = None
        self.texture_grad_ready = None
        self.texture_grad_route = None  # GradSync: the per-render texel-gradient target (several renders per step)
        self.test_colors = None  # eval-render test colours (gstex.py:309)
        # defer_texture (not in the reference; fused Adam on a HIP device): the texel parameter's Adam update of step k
        # (73 % of the parameters at cfg3) runs at step k+1's zero_grad() or render, before the raster forward, the first reader of
        # the texels -- at the pair-count read-back when there is one (the device runs it while the host waits), else
        # right before the raster forward.  Same updates in the same order on the same stream; the gradient is a
        # persistent buffer the raster forward zeroes (no per-step fill).  Readers of texture_dc outside the step go
        # through wait_texture() / texels(), which run a pending update.  (A side-stream texel update, overlapping
        # the next step's preprocessing and binning, measured no gain in rounds 2-3: the compute stream's kernels
        # slow down under the streaming update by what the overlap saves; removed in round 5.)
        self.defer_texture = bool(defer_texture) and fused_adam and self.device.type == "cuda"
        self._pending_tex = None
        self._pending_collective = False  # the pending update first waits for a GradSync collective
        # the texel-gradient sink is zeroed by the first differentiable raster forward after an optimizer step
        # (gstex_raster_fwd_zero), so several renders of one step still accumulate their texel gradients
        self._sink_fresh = True
        # pair_capacity (not in the reference; fused Adam on a HIP device): the training renders size their pair
        # buffers from an ops.PairCapacity instead of reading the pair total back to the host (gstex.py:1045-1052,
        # 1127), so a step has no host synchronisation.  Each step's renders write an overflow flag into
        # step_control[step % 8] (a device fp32 ring; gstex_amd.dist.GradSync replaces it by a slice of its flat
        # buffer, all-reduced with the gradients) that every Adam launch of the step reads (skip on overflow).
        # GSTEX_SYNC_PAIRS=1 restores the read-back.
        if pair_capacity is None:
            pair_capacity = os.environ.get("GSTEX_SYNC_PAIRS", "0") == "0"
        self.pairs = ops.PairCapacity(d) if (pair_capacity and fused_adam and self.device.type == "cuda") else None
        self.step_control = torch.zeros(8, device=d, dtype=torch.float32)
        self.skipped_steps = []  # steps whose update the pair-capacity guard skipped (found by _poll_pairs)
        # fused_step (not in the reference): the photometric training render as one C prologue call and one autograd
        # node (gstex_amd.fused) -- the same launches with ~0.23 ms less host time before the raster forward (the
        # device idles through that after a synchronisation); GSTEX_FUSED_STEP=0 restores the per-op render
        if fused_step is None:
            fused_step = os.environ.get("GSTEX_FUSED_STEP", "1") != "0"
        self.fused_step = bool(fused_step)
        self._tex_grad = None
        self._tex_grad_next = None
        self._cur_zeroed = self._next_zeroed = False
        if self.defer_texture:
            self._own_texture_grad()
        self._build_optimizer()

    def _own_texture_grad(self):
        # the persistent texel-gradient buffer (replaced by a flat-buffer slice when GradSync takes over).  With the
        # fused render a second one: step k's raster backward accumulates into one and zeroes the other
        # (gstex_raster_bwd_zero), which step k + 1 accumulates into, so no forward spends its grid zeroing 120 MB
        self._tex_grad = torch.zeros_like(self.texture_dc)
        # (not under GradSync, whose flat-buffer slice is the sink: the second buffer would never be used)
        self._tex_grad_next = (torch.zeros_like(self.texture_dc)
                               if self.fused_step and self.texture_grad_route is None else None)
        self._cur_zeroed = True  # the current buffer holds no gradient
        self._next_zeroed = self._tex_grad_next is not None
        self.texture_dc.grad = self._tex_grad
        self.texture_grad_sink = self._tex_grad

    def _double_buffered(self) -> bool:
        return (self._tex_grad_next is not None and self.texture_grad_route is None
                and self.texture_grad_sink is self._tex_grad)

    def _step_texels(self, buf, only, skip_flag):
        """The deferred texel update reading `buf` (the gradient buffer of the step it belongs to)."""
        keep = self.texture_dc.grad
        self.texture_dc.grad = buf
        try:
            self._step(only=only, skip_flag=skip_flag)
        finally:
            self.texture_dc.grad = keep

    @property
    def texture_grad_zeroed_by_update(self) -> bool:
        """The texel gradient buffer handed to the raster (texture_grad_sink) is zeroed by the raster forward
        (gstex_raster_fwd_zero) before the backward accumulates into it: a gradient-buffer owner
        (gstex_amd.dist.GradSync) must not fill that slice itself (with the deferred texel update, defer_texture, that
        fill would also pre-empt the update still reading it)."""
        return True

    def reset_texture_grad(self):
        """Zero the texel-gradient sink lazily: the next differentiable render's raster forward zeroes it before its
        backward accumulates (gstex_raster_fwd_zero).  Called by zero_grad() and by gstex_amd.dist.GradSync.zero(), so
        a gradient left by a backward whose step was skipped never leaks into the next step."""
        self._sink_fresh = True

    def _skip_flag(self):
        """The current step's guard flag (1-element view of step_control) for its Adam launches, or None."""
        if self.pairs is None:
            return None
        k = self.step % 8
        return self.step_control[k:k + 1]

    def _poll_pairs(self):
        """Pair totals of finished renders (non-blocking): grows the capacity, records skipped steps."""
        if self.pairs is not None and self.pairs.poll():
            import warnings

            new = self.pairs.overflows[len(self.skipped_steps):]
            self.skipped_steps.extend(new)
            warnings.warn(f"GStexTrainer: the pair total of step(s) {new} exceeded the pair capacity; their updates "
                          f"were skipped on the device and the capacity grew to {self.pairs.capacity}")

    def _run_pending_texture(self):
        fn, self._pending_tex = self._pending_tex, None
        if fn is not None:
            fn()

    def wait_texture(self):
        """Order the current stream after the pending texel update (defer_texture): it is enqueued now."""
        self._run_pending_texture()

    def texels(self) -> torch.Tensor:
        """The texel store (SH-DC values) for readers outside the step (export, average_colors, viewers): runs a
        pending deferred update first (defer_texture), so no reader depends on remembering wait_texture()."""
        self.wait_texture()
        return self.texture_dc.detach()

    # ------------------------------------------------------------------ parameters
    def param_groups(self):
        return {
            "xyz": [self.means],
            "features_dc": [self.features_dc],
            "features_rest": [self.features_rest],
            "opacity": [self.opacities],
            "scaling": [self.scales],
            "rotation": [self.quats],
            "texture_dc": [self.texture_dc],
        }

    def parameters(self):
        return [p for ps in self.param_groups().values() for p in ps]

    def _build_optimizer(self):
        groups = [{"params": ps, "lr": LRS[name], "name": name} for name, ps in self.param_groups().items()]
        if self.fused_adam:
            self.optimizer = FusedAdam(groups, eps=1e-15)
        else:
            self.optimizer = torch.optim.Adam(groups, eps=1e-15, foreach=True)

    # ------------------------------------------------------------------ forward
    def render(self, view: View, sh_degree_now: int | None = None, composite: bool = True, geometry: bool | None = None):
        """get_outputs (gstex.py:992-1236), training branch.  geometry: render depth / distortion / normal (default:
        the trainer's geometry_outputs).  sh_degree_now: default min(step // sh_degree_interval, sh_degree), as
        get_outputs evaluates it in training and eval alike (gstex.py:1103)."""
        means = self.means
        deg = self.sh_degree_now() if sh_degree_now is None else sh_degree_now
        if self._pending_tex is not None and not self._pending_collective and self.pairs is not None:
            # the deferred texel update first (read-back-free step: there is no pair-count wait to fill): ~90 us of
            # streaming work the device starts on while the host enqueues the step's short preprocessing and binning
            # launches, instead of idling through them after a synchronisation (the bench's first timed step); it only
            # has to land before the raster forward, the first reader of the texels
            self._run_pending_texture()
        if self._fused_ok(composite, geometry):
            return self._render_fused(view, deg)
        if self.fused_activations:  # one HIP launch each way (gstex_amd.activations)
            quats, scales, opacities, uv0, umap, vmap, viewdirs = activate(
                means, self.quats, self.scales, self.opacities, self.mappings, view.campos)
        else:
            quats = self.quats / self.quats.norm(dim=-1, keepdim=True)
            s = torch.exp(self.scales[:, :-1]).clamp(min=1e-9)
            scales = torch.cat([s, 1e-5 * s.mean(dim=-1, keepdim=True).detach()], dim=-1)
            opacities = torch.sigmoid(self.opacities)
            uv0, umap, vmap = get_uv_mapping(quats, self.mappings)
            viewdirs = means.detach() - view.c2w[:3, 3]
            viewdirs = viewdirs / viewdirs.norm(dim=-1, keepdim=True)
        if self.fix_init and self.sh_degree > 0:
            viewdirs = torch.stack([viewdirs[:, 0], -viewdirs[:, 2], viewdirs[:, 1]], -1)
        intr = (view.fx, view.fy, view.cx, view.cy)
        # project_points / get_aabb_2d / get_num_tiles_hit_2d (gstex.py:1077-1080) in one launch; the centre
        # gradient is chained inside the raster backward (fold_aabb below), the depths only order the tile lists
        depths, centers, extents, nth = ops.preprocess(means, scales, 1, quats, view.viewmat, intr, view.H, view.W)
        n = self.means.shape[0]
        if self.sh_degree > 0:
            if self.fused_activations:  # the zeroed DC term (gstex.py:1100) without the cat
                rgbs = sh_rest(deg, viewdirs, self.features_rest)
            else:
                colors = torch.cat([torch.zeros_like(self.features_dc[:, None, :]), self.features_rest], dim=1)
                rgbs = ops.spherical_harmonics(deg, viewdirs, colors)
        else:
            rgbs = torch.sigmoid(self.features_dc)
        # SH2RGB(texture_dc) (gstex.py:1119) applied by the raster on read instead of materialised
        texture = self.texture_dc
        # the deferred texel update: while the host waits for the pair count (one GPU: it fills the device's idle time
        # there), or -- when it first waits for its data-parallel collective (GradSync) -- right before the raster
        # forward, so that the binning's placement and sort do not queue behind that wait
        pend = self._pending_tex is not None
        late = pend and self._pending_collective
        if self.texture_grad_route is not None and torch.is_grad_enabled():
            sink, zero_sink, on_grad = self.texture_grad_route(self._sink_fresh)
        else:
            sink, zero_sink, on_grad = self.texture_grad_sink, self._sink_fresh, self.texture_grad_ready
        guard = None
        if self.pairs is not None and torch.is_grad_enabled():
            self._poll_pairs()
            guard = (self.pairs, self._skip_flag(), self._sink_fresh, self.step)
        img, depth, reg, alpha, tex, normal = ops.texture_gaussians(
            (n, 1, 3), self.texture_dims, centers, extents, depths, nth, rgbs, opacities, means, scales, 1, quats,
            uv0, umap, vmap, texture, view.viewmat, view.c2w, view.fx, view.fy, view.cx, view.cy, view.H, view.W,
            ops.BLOCK_WIDTH, self.settings, background=self._bg_zero,
            texture_transform=(SH_C0, 0.5), fold_aabb=True,  # centers come from get_aabb_2d just above
            geometry_outputs=self.geometry_outputs if geometry is None else geometry,
            texture_grad_sink=sink, zero_texture_grad_sink=zero_sink, on_texture_grad=on_grad,
            texture_ready=self._run_pending_texture if late else None,
            before_pair_wait=self._run_pending_texture if pend and not late else None,
            pair_guard=guard)
        if torch.is_grad_enabled():
            self._sink_fresh = False  # zeroed by this forward: further renders before the step accumulate on top
            self._cur_zeroed = False
        out = dict(img=img, tex=tex, depth=depth, reg=reg, alpha=alpha, normal=normal)
        if composite:
            out["rgb"] = torch.clamp(img + tex[:, :, 0:3] + (1 - alpha[:, :, None]) * self.background[None, None, :],
                                     0.0, 1.0)
        return out

    def _fused_ok(self, composite: bool, geometry) -> bool:
        """Whether render() takes gstex_amd.fused's path (see its docstring for why each condition is there)."""
        return (self.fused_step and not composite and not (self.geometry_outputs if geometry is None else geometry)
                and self.fused_activations and self.sh_degree > 0 and not self.fix_init
                and self.pairs is not None and self.pairs.capacity > 0 and self.texture_grad_sink is not None
                and torch.is_grad_enabled() and not torch.are_deterministic_algorithms_enabled()
                and not torch.cuda.is_current_stream_capturing())

    def _render_fused(self, view: View, deg: int):
        from . import fused

        # the texel-gradient target as in the per-op render: GradSync's route (the flat buffer's slice, or its side
        # buffer once the tail's collective is on the wire) or the trainer's own sink
        if self.texture_grad_route is not None:
            sink, zero_sink, on_grad = self.texture_grad_route(self._sink_fresh)
        else:
            sink, zero_sink, on_grad = self.texture_grad_sink, self._sink_fresh, self.texture_grad_ready
        # a deferred texel update that first waits for its collective (GradSync) runs right before the raster forward
        late = self._run_pending_texture if self._pending_tex is not None and self._pending_collective else None
        zero_next = None
        if self._double_buffered():
            zero_sink = zero_sink and not self._cur_zeroed  # (zeroed by the previous step's raster backward)
            zero_next = None if self._next_zeroed else self._tex_grad_next  # this backward zeroes the other buffer
        self._poll_pairs()
        img, alpha, tex = fused.train_render(self, view, deg, sink, zero_sink, self._sink_fresh, on_grad, late,
                                             zero_next)
        self._sink_fresh = False
        self._cur_zeroed = False
        z = ops._zero_scalar(self.device)  # not rendered: read-only zeros without gradient, as the per-op path
        H, W = int(view.H), int(view.W)
        return dict(img=img, tex=tex, depth=z.expand(H, W), reg=z.expand(H, W), alpha=alpha,
                    normal=z.expand(H, W, 3))

    @torch.no_grad()
    def eval_render(self, view: View, edit_texture: torch.Tensor | None = None):
        """The reference's eval render (get_outputs with extra_stuff, gstex.py:1086-1203): a 6-channel texture
        [SH2RGB(texture_dc), 0, 0, 0] and three raster calls -- the image, the test-colour render with
        thresholded opacities (test_img / uv_im) and the settings | 1 << 15 render (edit_img, clean normals).
        Same outputs (tests/test_gpu_eval.py checks them against those three 6-channel calls), computed with one
        binning and the 3-channel raster (below)."""
        self.wait_texture()
        means = self.means
        quats, scales, opacities, uv0, umap, vmap, viewdirs = activate(
            means, self.quats, self.scales, self.opacities, self.mappings, view.campos)
        if self.fix_init and self.sh_degree > 0:
            viewdirs = torch.stack([viewdirs[:, 0], -viewdirs[:, 2], viewdirs[:, 1]], -1)
        intr = (view.fx, view.fy, view.cx, view.cy)
        _, depths = ops.project_points(means, view.viewmat, intr)
        centers, extents = ops.get_aabb_2d(means, scales, 1, quats, view.viewmat, intr)
        nth = ops.get_num_tiles_hit_2d(centers, extents, view.H, view.W, ops.BLOCK_WIDTH)
        n = means.shape[0]
        rgbs = (sh_rest(self.sh_degree_now(), viewdirs, self.features_rest) if self.sh_degree > 0
                else torch.sigmoid(self.features_dc))
        if self.test_colors is None or self.test_colors.shape[0] != n:
            g = torch.Generator(device="cpu").manual_seed(0)
            self.test_colors = torch.rand((n, 3), generator=g).to(means.device)  # gstex.py:309
        bgz = self._bg_zero
        # the three calls share one geometry: binned and sorted once.  The reference's 6-channel texture is
        # [SH2RGB(texture_dc), 0, 0, 0] for the first call and [edit_texture or 0, 0, 0, 0] for the other two; a
        # zero texel contributes exactly 0, so each call runs the 3-channel raster (SH2RGB as texture_transform,
        # the all-zero texture as transform (0, 0)) and channels 3..5 of its texture output are zeros -- the same
        # outputs without materialising two 6-channel copies of the texel store
        bins = ops.bin_gaussians(centers, extents, depths, nth, view.H, view.W)

        def tg(cr, tex, transform, co, st):
            return ops.texture_gaussians(
                (n, 1, 3), self.texture_dims, centers, extents, depths, nth, cr, co, means, scales, 1, quats, uv0,
                umap, vmap, tex, view.viewmat, view.c2w, view.fx, view.fy, view.cx, view.cy, view.H, view.W,
                ops.BLOCK_WIDTH, st, background=bgz, texture_transform=transform, binning=bins)

        img, depth, reg, alpha, tex, normal = tg(rgbs, self.texture_dc, (SH_C0, 0.5), opacities, self.settings)
        upd, upd_tf = (edit_texture, None) if edit_texture is not None else (self.texture_dc, (0.0, 0.0))
        test_op = opacities.clone()
        test_op[test_op <= 0.5] = 0.0
        test_op[test_op > 0.2] = 1.0
        t_out = tg(self.test_colors, upd, upd_tf, test_op, self.settings)
        if edit_texture is not None:
            n_edit, n_unit = tg(self.test_colors, upd, upd_tf, opacities, self.settings | (1 << 15))[4:6]
        else:
            # the settings | 1 << 15 call has the first call's geometry and weights: its texture output is the zero
            # texture's (0) and its normal is the first call's accumulated normal as a unit vector (0 where none),
            # the same fp32 operations as the kernel's bit-15 epilogue -- no third raster pass
            n2 = (normal[..., 0] * normal[..., 0] + normal[..., 1] * normal[..., 1]) + normal[..., 2] * normal[..., 2]
            inv = torch.where(n2 > 0, 1.0 / torch.sqrt(n2), torch.zeros_like(n2))
            n_edit, n_unit = None, normal * inv[..., None]
        zeros3 = torch.zeros_like(img)  # texture channels 3..5 of every call
        bg = self.background[None, None, :]
        rgb = torch.clamp(img + tex[..., 0:3] + (1 - alpha[..., None]) * bg, 0.0, 1.0)
        edit_tex_img = n_edit[..., :3] if n_edit is not None else zeros3
        return dict(rgb=rgb, depth=depth, alpha=alpha, normal=normal,
                    test_img=t_out[0] + (1 - t_out[3][..., None]) * bg,
                    uv_im=torch.clamp(zeros3 + (1 - t_out[3][..., None]) * bg, 0.0, 1.0),
                    edit_img=torch.clamp(img + edit_tex_img + (1 - alpha[..., None]) * bg, 0.0, 1.0),
                    clean_normal_img=torch.clamp(0.5 * (n_unit + 1) + (1 - alpha[..., None]) * bg, 0.0, 1.0))

    def loss(self, rgb: torch.Tensor, gt: torch.Tensor, ssim_lambda: float = 0.2) -> torch.Tensor:
        l1 = torch.abs(gt - rgb).mean()
        sim = 1 - ssim(gt.permute(2, 0, 1)[None], rgb.permute(2, 0, 1)[None])
        return (1 - ssim_lambda) * l1 + ssim_lambda * sim

    def sh_degree_now(self) -> int:
        """The SH degree ramp of the reference: min(step // sh_degree_interval, sh_degree) (gstex.py:1103)."""
        return min(self.step // self.sh_degree_interval, self.sh_degree)

    def forward_backward(self, view: View, gt: torch.Tensor) -> StepOutput:
        lam_n, lam_r = scheduled(self.lambda_normal, self.step), scheduled(self.lambda_reg, self.step)
        geo = lam_n != 0.0 or lam_r != 0.0
        out = self.render(view, sh_degree_now=self.sh_degree_now(), composite=not self.fused_loss,
                          geometry=True if geo else None)
        if self.fused_loss:  # composite + clamp + L1/SSIM in one HIP launch pair (gstex_amd.loss)
            loss, rgb = photometric_loss(out["img"], out["tex"], out["alpha"], self.background, gt.contiguous())
        else:
            rgb = out["rgb"]
            loss = self.loss(rgb, gt)
        if geo:
            # gstex.py:1218-1222: the depth-derived normal (detached) when use_normal_loss, else the rendered normal
            est = (depth_to_normal(out["depth"], view.viewmat, view.c2w, view.fx, view.fy, view.cx, view.cy).detach()
                   if self.use_normal_loss else out["normal"])
            loss = loss + geometry_loss(out["alpha"], out["normal"], est, out["reg"], lam_n, lam_r)
        loss.backward(self._one)  # (a cached seed: no per-step fill launch for the implicit ones_like)
        return StepOutput(loss.detach(), rgb.detach())

    def optimizer_step(self, sync=None):
        """The Adam step.  With a gstex_amd.dist.GradSync `sync` (data-parallel training) the gradient exchange is part
        of the step: the texel group is updated as soon as its collective lands, overlapping the head's collective,
        and the 1 / world averaging rides in the fused update (GradSync.all_reduce_and_step); otherwise call
        sync.all_reduce() before this."""
        self._sink_fresh = True  # the next step's first render zeroes the texel-gradient sink
        sf = self._skip_flag()  # this step's pair-capacity guard (None without pair_capacity)
        if self.defer_texture:
            self._run_pending_texture()  # (two steps without a render in between)
            tex = {id(self.texture_dc)}
            if sync is not None:
                # the texel update in pieces, each as soon as its piece of the collective has landed (GradSync)
                rng = (lambda s, lo, hi, first: self.optimizer.step_range(self.texture_dc, lo, hi, first,
                                                                          grad_scale=s, skip_flag=sf)) \
                    if self.fused_adam else None
                self._pending_tex = sync.all_reduce_and_step(
                    lambda s: self.optimizer.step(only=tex, grad_scale=s, skip_flag=sf),
                    lambda s: self.optimizer.step(skip=tex, grad_scale=s, skip_flag=sf), defer_tail=True,
                    step_tail_range=rng)
                self._pending_collective = True
            else:
                self._step(skip=tex, skip_flag=sf)
                buf = self.texture_dc.grad
                self._pending_tex = lambda: self._step_texels(buf, tex, sf)
                self._pending_collective = False
                if self._double_buffered():
                    # the next step accumulates into the other buffer (zeroed by this step's raster backward, or
                    # else by the next forward); the pending update reads this one
                    self._tex_grad, self._tex_grad_next = self._tex_grad_next, self._tex_grad
                    self._cur_zeroed, self._next_zeroed = self._next_zeroed, False
                    self.texture_dc.grad = self._tex_grad
                    self.texture_grad_sink = self._tex_grad
            self.step += 1
            return
        if sync is not None and self.fused_adam:
            tex = {id(self.texture_dc)}
            sync.all_reduce_and_step(lambda s: self.optimizer.step(only=tex, grad_scale=s, skip_flag=sf),
                                     lambda s: self.optimizer.step(skip=tex, grad_scale=s, skip_flag=sf))
            self.step += 1
            return
        if sync is not None:
            sync.all_reduce()
        self._step(skip_flag=sf)
        self.step += 1

    def _step(self, **kw):
        """optimizer.step with the fused optimizer's extensions (skip_flag is None without pair_capacity, which needs
        the fused Adam)."""
        if kw.get("skip_flag") is None:
            kw.pop("skip_flag", None)
        self.optimizer.step(**kw)

    def zero_grad(self, set_to_none: bool = True):
        """Optimizers.zero_grad_all (engine/optimizers.py): torch's default set_to_none=True, so backward
        writes fresh gradients instead of accumulating into zero-filled ones.  Keep set_to_none=False
        when .grad tensors are views of a flat buffer (gstex_amd.dist.GradSync zeroes that instead).  With
        defer_texture the texel gradient buffer is kept (the raster forward zeroes it), and the previous step's deferred
        texel update is enqueued here, first: it reads that buffer (which set_to_none=False would otherwise zero under
        it), and a step that starts on an idle device -- after a synchronisation -- gets its first long kernel without
        waiting for the host to reach the render (the launch order on the stream is the same as from render())."""
        if self._pending_tex is not None and not self._pending_collective:
            self._run_pending_texture()
        self.reset_texture_grad()
        if self.defer_texture:
            keep = self.texture_dc.grad
            self.optimizer.zero_grad(set_to_none=set_to_none)
            self.texture_dc.grad = keep
            return
        self.optimizer.zero_grad(set_to_none=set_to_none)

    # ------------------------------------------------------------------ rechart
    @torch.no_grad()
    def recharge(self):
        """retexture_after (gstex.py:890-895): rebuild the charts from the current scales, resample the texels
        onto the new grid (texture_sample, JaggedTexture.init_from_dims, jagged_texture.py:116-143) and reset the
        texture Adam moments (reshape_in_optim, gstex.py:799-826: exp_avg / exp_avg_sq zeroed, step kept).

        The texel store is reused in place while the new charts fit its capacity (jagged_texture.py:45-64:
        adjust_texture_size only ever grows it), so the Parameter, its optimizer entry and any flat gradient
        buffer built over it (gstex_amd.dist.GradSync) stay valid; only a growth replaces the Parameter."""
        self.wait_texture()
        new_dims, mappings, _ = build_charts(self.scales.detach(), self.pixel_num)
        n_new = int((new_dims[:, 0].long() * new_dims[:, 1].long()).sum())
        ids, uv = texture_dims_to_query(new_dims)
        query = self.texture_dims[ids].contiguous()
        new_tex = ops.texture_sample((1, 1, 3), query, self.texture_dc.detach(), uv.contiguous())
        old = self.texture_dc
        cap = old.shape[0]
        if n_new > cap:  # adjust_texture_size: grow with zero rows (jagged_texture.py:53-64)
            store = torch.cat([old.detach(), old.new_zeros((n_new - cap, old.shape[1]))], 0)
            self.texture_dc = torch.nn.Parameter(store)
            for g in self.optimizer.param_groups:
                if g["name"] == "texture_dc":
                    g["params"] = [self.texture_dc]
            st = self.optimizer.state.pop(old, None)
            if st:
                self.optimizer.state[self.texture_dc] = {
                    "step": st.get("step", 0),
                    "exp_avg": torch.zeros_like(self.texture_dc),
                    "exp_avg_sq": torch.zeros_like(self.texture_dc),
                }
            if self.defer_texture:  # a fresh persistent gradient buffer (GradSync replaces it)
                self._own_texture_grad()
        else:
            st = self.optimizer.state.get(old)
            if st:
                st["exp_avg"].zero_()
                st["exp_avg_sq"].zero_()
        self.texture_dc.data[:n_new] = new_tex
        self.texture_dims = new_dims.contiguous()
        self.n_texels = n_new
        self.mappings.copy_(mappings)
        return new_dims
