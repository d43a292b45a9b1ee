#!/usr/bin/env python3
"""Forward workgroup balance at cfg3: per 256-position segment of a tile, the 4 quadrant waves' visit counts (the
unit costs the forward writes into its aux record).  A 4-wave workgroup that synchronises per batch runs a segment
for at least max_q(count); independent waves would need mean_q.  Prints sum(max) / sum(mean)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gstex_amd import ops  # noqa: E402
from gstex_amd.scene import make_scene, sphere_view  # noqa: E402

dev = torch.device("cuda", 0)
sc = make_scene(200_000, 1e7, seed=42, opacity=0.1)
v = sphere_view(0, 800, 800).to(dev)
means, scales, quats, opac = [t.to(dev) for t in sc.activated()]
uv0, umap, vmap = [t.to(dev) for t in sc.uv_mapping()]
rgbs = torch.rand((sc.n, 3), device=dev).requires_grad_(True)
tex = sc.texture.to(dev)
intr = (v.fx, v.fy, v.cx, v.cy)
_, depths = ops.project_points(means, v.viewmat, intr)
c, e = ops.get_aabb_2d(means, scales, 1, quats, v.viewmat, intr)
nth = ops.get_num_tiles_hit_2d(c, e, 800, 800, 16)
outs = ops.texture_gaussians((sc.n, 1, 3), sc.texture_dims.to(dev), c, e, depths, nth, rgbs, opac, means, scales, 1,
                             quats, uv0, umap, vmap, tex, v.viewmat, v.c2w, v.fx, v.fy, v.cx, v.cy, 800, 800, 16,
                             (1 << 9) | (1 << 10), background=None, geometry_outputs=False)
torch.cuda.synchronize()
aux = outs[0].grad_fn.aux.cpu().numpy()
n_isect = int(nth.sum())
n_tiles = 50 * 50
al = lambda x: (x + 255) & ~255
masks = al(((n_isect + 63) // 64 + n_tiles + 1) * 4 * 8)
n_slots = (n_isect + 255) // 256 + n_tiles + 1
cost = aux[masks:masks + n_slots * 16].view(np.int32).reshape(n_slots, 4) & 0xFFFFFF
live = cost.max(1) > 0
mx, mean = cost.max(1)[live].sum(), cost.mean(1)[live].sum()
print(f"segments {live.sum()}, visits {cost.sum()}, sum max {mx}, sum mean {mean:.0f}, ratio {mx / mean:.3f}")
