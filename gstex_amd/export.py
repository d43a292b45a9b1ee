"""GStex parameter export/import in the reference's NPZ wire format.

``export_npz`` writes exactly the arrays of ``ExportGStexNpz`` (nerfstudio/scripts/exporter.py:78-105):
xyz, features_rest, opacity, scaling, rotation, texture_dc, texture_dims, mappings (parameters in
their stored, pre-activation form; texture_dc holds SH-DC values, gstex.py:1119).  ``trainer_from_npz``
rebuilds a ``GStexTrainer`` from such a file bit-exactly (features_dc, which the exporter omits, is zero:
under SH colour the DC term is replaced by the texture, gstex.py:1100).  ``average_colors`` is
``GStexModel.get_average_colors`` (gstex.py:714-726), used by the reference's PLY export.
"""
from __future__ import annotations

import numpy as np
import torch

from .charts import SH2RGB

NPZ_KEYS = ("xyz", "features_rest", "opacity", "scaling", "rotation", "texture_dc", "texture_dims", "mappings")


def export_npz(trainer, path) -> None:
    if hasattr(trainer, "wait_texture"):  # defer_texture: the pending texel update must run before the read
        trainer.wait_texture()
    params = {
        "xyz": trainer.means,
        "features_rest": trainer.features_rest,
        "opacity": trainer.opacities,
        "scaling": trainer.scales,
        "rotation": trainer.quats,
        "texture_dc": trainer.texture_dc,
        "texture_dims": trainer.texture_dims,
        "mappings": trainer.mappings,
    }
    np.savez(path, **{k: v.detach().cpu().numpy() for k, v in params.items()})


def load_npz(path) -> dict:
    """The NPZ arrays as CPU tensors (no pickle: allow_pickle=False)."""
    with np.load(path, allow_pickle=False) as z:
        missing = [k for k in NPZ_KEYS if k not in z.files]
        if missing:
            raise KeyError(f"{path}: not a GStex NPZ export, missing {missing}")
        return {k: torch.from_numpy(np.array(z[k])) for k in NPZ_KEYS}


def average_colors(texture_dc: torch.Tensor, texture_dims: torch.Tensor, sh_degree: int = 3) -> torch.Tensor:
    """Per-splat mean texel colour (gstex.py:714-726): SH2RGB (sigmoid without SH) of each splat's
    h*w texels, averaged."""
    n = texture_dims.shape[0]
    hws = (texture_dims[:, 0] * texture_dims[:, 1]).long()
    ids = torch.repeat_interleave(torch.arange(n, device=texture_dims.device), hws)
    tex = texture_dc[: ids.numel()]
    tex = SH2RGB(tex) if sh_degree > 0 else torch.sigmoid(tex)
    avg = torch.zeros((n, tex.shape[-1]), device=tex.device, dtype=torch.float32)
    return torch.index_add(avg, 0, ids, tex) / hws.float()[:, None]


def trainer_from_npz(path, device, **trainer_kwargs):
    """A GStexTrainer holding exactly the exported parameters (fresh optimizer state)."""
    from .model import GStexTrainer
    from .scene import Scene

    d = load_npz(path)
    n = d["xyz"].shape[0]
    zeros = torch.zeros((n, 3), dtype=torch.float32)
    scene = Scene(means=d["xyz"], log_scales=d["scaling"], quats=d["rotation"], opacity_logits=d["opacity"],
                  features_dc=zeros, features_rest=d["features_rest"], rgbs=zeros,
                  texture_dims=d["texture_dims"].to(torch.int32), mappings=d["mappings"],
                  texture=SH2RGB(d["texture_dc"]), pixel_scale=float("nan"))
    tr = GStexTrainer(scene, device, pixel_num=float(d["texture_dc"].shape[0]), **trainer_kwargs)
    with torch.no_grad():  # the raster-space round trip SH2RGB -> (x - 0.5) / C0 is not exact: copy the DC
        tr.texture_dc.copy_(d["texture_dc"].to(tr.device))
    return tr
