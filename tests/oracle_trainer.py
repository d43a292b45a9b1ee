"""An oracle-driven GStex trainer on the CPU (test infrastructure, the checker of tests/test_gpu_trajectory.py).

The same training step as gstex_amd.model.GStexTrainer (the reference's, gstex.py:992-1236 + 1277-1322 +
engine/optimizers.py), with every rasterizer op replaced by the CPU oracle (oracle/raster.py) in fp32 and its backward
by torch autograd through the oracle, and the fused HIP kernels by eager torch:
  * activations gstex.py:1059-1066, UV frames :975-990 (detached), SH colour with the DC zeroed :1099-1114
    (oracle.spherical_harmonics), texels read as SH2RGB(texture_dc) :1119;
  * get_aabb_2d / project_points / get_num_tiles_hit_2d (oracle), texture_gaussians (oracle.rasterize, its fp32
    re-evaluation under the fp32 decisions, differentiable), settings (1 << 9) | (1 << 10), zero raster background;
  * composite :1204-1205 with the trainer's background and the loss 0.8 L1 + 0.2 (1 - SSIM) :1301-1322
    (gstex_amd.model.ssim, the eager pytorch_msssim restatement);
  * per-group torch.optim.Adam(eps=1e-15) with the gstex-blender-nvs learning rates (gstex_configs.py:207-244);
  * recharge: build_charts of the current scales, the texels resampled at the new charts' query uvs
    (oracle.texture_sample, jagged_texture.py:116-143), the texel moments reset, the store grown when needed
    (gstex.py:799-826, 890-895).
"""
from __future__ import annotations

import torch

from gstex_amd.charts import SH2RGB, build_charts, get_uv_mapping, texture_dims_to_query
from gstex_amd.model import DEFAULT_SETTINGS, LRS, ssim
from gstex_amd.scene import Scene, View
from oracle import raster as O


class OracleTrainer:
    def __init__(self, scene: Scene, background=(1.0, 1.0, 1.0), start_step: int = 3000, sh_degree: int = 3,
                 sh_degree_interval: int = 1000):
        P = lambda t: torch.nn.Parameter(t.detach().clone().float())  # noqa: E731
        self.means, self.scales, self.quats = P(scene.means), P(scene.log_scales), P(scene.quats)
        self.opacities = P(scene.opacity_logits)
        self.features_dc, self.features_rest = P(scene.features_dc), P(scene.features_rest)
        self.texture_dc = P((scene.texture[:, :3] - 0.5) / 0.28209479177387814)
        self.texture_dims = scene.texture_dims.clone()
        self.mappings = scene.mappings.clone()
        self.pixel_num = float(scene.texture.shape[0])
        self.background = torch.tensor(background, dtype=torch.float32)
        self.step = start_step
        self.sh_degree, self.sh_degree_interval = sh_degree, sh_degree_interval
        groups = [{"params": ps, "lr": LRS[name], "name": name} for name, ps in self.param_groups().items()]
        self.optimizer = torch.optim.Adam(groups, eps=1e-15)

    def param_groups(self):
        return {"xyz": [self.means], "features_dc": [self.features_dc], "features_rest": [self.features_rest],
                "opacity": [self.opacities], "scaling": [self.scales], "rotation": [self.quats],
                "texture_dc": [self.texture_dc]}

    def parameters(self):
        return [p for ps in self.param_groups().values() for p in ps]

    def sh_degree_now(self) -> int:
        """min(step // sh_degree_interval, sh_degree) (gstex.py:1103)."""
        return min(self.step // self.sh_degree_interval, self.sh_degree)

    def render(self, view: View):
        quats = self.quats / self.quats.norm(dim=-1, keepdim=True)
        s = torch.exp(self.scales[:, :-1]).clamp(min=1e-9)
        scales = torch.cat([s, 1e-5 * s.mean(dim=-1, keepdim=True).detach()], dim=-1)
        opac = torch.sigmoid(self.opacities)
        uv0, umap, vmap = get_uv_mapping(quats, self.mappings)
        campos = view.c2w[:3, 3]
        viewdirs = self.means.detach() - campos
        viewdirs = viewdirs / viewdirs.norm(dim=-1, keepdim=True)
        cam = O.Camera(view.viewmat, view.fx, view.fy, view.cx, view.cy, view.H, view.W, 16, campos)
        centers, extents = O.aabb_2d(self.means, scales, 1.0, quats, cam)
        _, depths = O.project_points(self.means.detach(), cam)
        deg = self.sh_degree_now()
        coeffs = torch.cat([torch.zeros_like(self.features_rest[:, :1, :]), self.features_rest], 1)
        rgbs = O.spherical_harmonics(deg, viewdirs, coeffs)
        texture = SH2RGB(self.texture_dc)
        inp = O.RasterInputs(self.texture_dims, centers, extents, depths.detach(), rgbs, opac, self.means, scales, 1.0,
                             quats, uv0, umap, vmap, texture, cam, DEFAULT_SETTINGS, None)
        _, out, _ = O.rasterize(inp, grad_dtype=torch.float32)
        rgb = torch.clamp(out["img"] + out["tex"][:, :, 0:3] + (1 - out["alpha"][:, :, None]) * self.background, 0.0,
                          1.0)
        return rgb

    def forward_backward(self, view: View, gt: torch.Tensor) -> float:
        rgb = self.render(view)
        l1 = torch.abs(gt - rgb).mean()
        sim = 1 - ssim(gt.permute(2, 0, 1)[None], rgb.permute(2, 0, 1)[None])
        loss = 0.8 * l1 + 0.2 * sim
        loss.backward()
        return float(loss.detach())

    def zero_grad(self):
        self.optimizer.zero_grad(set_to_none=True)

    def optimizer_step(self):
        self.optimizer.step()
        self.step += 1

    @torch.no_grad()
    def recharge(self):
        new_dims, mappings, _ = build_charts(self.scales.detach(), self.pixel_num)
        n_new = int((new_dims[:, 0].long() * new_dims[:, 1].long()).sum())
        ids, uv = texture_dims_to_query(new_dims)
        new_tex = O.texture_sample(self.texture_dims[ids].contiguous(), self.texture_dc.detach(), uv.contiguous())
        old = self.texture_dc
        cap = old.shape[0]
        st = self.optimizer.state.get(old)
        if n_new > cap:
            store = torch.cat([old.detach(), old.new_zeros((n_new - cap, old.shape[1]))], 0)
            self.texture_dc = torch.nn.Parameter(store)
            for g in self.optimizer.param_groups:
                if g["name"] == "texture_dc":
                    g["params"] = [self.texture_dc]
            self.optimizer.state.pop(old, None)
            if st:
                self.optimizer.state[self.texture_dc] = {"step": st["step"],
                                                         "exp_avg": torch.zeros_like(self.texture_dc),
                                                         "exp_avg_sq": torch.zeros_like(self.texture_dc)}
        elif st:
            st["exp_avg"].zero_()
            st["exp_avg_sq"].zero_()
        self.texture_dc.data[:n_new] = new_tex
        self.texture_dims = new_dims.contiguous()
        self.mappings.copy_(mappings)
