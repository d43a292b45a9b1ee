#!/usr/bin/env python3
"""Backward visit counts at cfg3 if a backward wave covered two 8x8 quadrants of a tile (two pixels per lane):
per (tile, quadrant) the forward's cull bits clipped to the quadrant's last contributor are the visits a quadrant
wave walks today; a pair wave walks the union of its two quadrants' bits (the per-visit fixed work -- record read,
reduce, accumulator atomic, texel flush -- once per union visit, the per-pixel work once per quadrant visit).
Prints the quadrant visits and the unions for the horizontal ({0,1},{2,3}) and vertical ({0,2},{1,3}) pairings."""
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
intr = (v.fx, v.fy, v.cx, v.cy)
_, depths = ops.project_points(means, v.viewmat, intr)
c, e = ops.get_aabb_2d(means, scales, 1, quats, v.viewmat, intr)
nth = ops.get_num_tiles_hit_2d(c, e, 800, 800, 16)
outs = ops.texture_gaussians((sc.n, 1, 3), sc.texture_dims.to(dev), c, e, depths, nth, rgbs, opac, means, scales, 1,
                             quats, uv0, umap, vmap, sc.texture.to(dev), v.viewmat, v.c2w, v.fx, v.fy, v.cx, v.cy,
                             800, 800, 16, (1 << 9) | (1 << 10), background=None, geometry_outputs=False)
torch.cuda.synchronize()
gf = outs[0].grad_fn
saved = gf.saved_tensors
tile_ranges = saved[9].cpu().numpy().reshape(-1, 2)
state = saved[14].cpu().numpy().reshape(800, 800, 4)
last = state[..., 3].copy().view(np.int32)
aux = gf.aux.cpu().numpy()
n_tiles = tile_ranges.shape[0]
tiles_x = 50
masks = aux[:(((int(nth.sum()) + 63) // 64 + n_tiles + 1) * 4 * 8)].view(np.uint64)

quad_visits = np.zeros(4, np.int64)
union = {"h": 0, "v": 0, "all4": 0}
for t in range(n_tiles):
    s, e_ = tile_ranges[t]
    if e_ <= s:
        continue
    tx, ty = t % tiles_x, t // tiles_x
    nw = (e_ - s + 63) // 64
    base = (s + 63) // 64 + t
    words = masks[(base * 4):(base + nw) * 4].reshape(nw, 4).copy()
    pos = np.arange(nw, dtype=np.int64)[:, None] * 64 + np.arange(64, dtype=np.int64)[None, :]
    bits = ((words[:, :, None] >> np.arange(64, dtype=np.uint64)[None, None, :]) & np.uint64(1)).astype(bool)
    bits = bits.transpose(1, 0, 2).reshape(4, -1)  # [quad][position]
    pos = pos.reshape(-1)
    for q in range(4):
        ox, oy = (q & 1) * 8, (q >> 1) * 8
        blk = last[ty * 16 + oy:ty * 16 + oy + 8, tx * 16 + ox:tx * 16 + ox + 8]
        wl = int(blk.max()) if blk.size else -1
        bits[q] &= pos <= wl
    quad_visits += bits.sum(1)
    union["h"] += (bits[0] | bits[1]).sum() + (bits[2] | bits[3]).sum()
    union["v"] += (bits[0] | bits[2]).sum() + (bits[1] | bits[3]).sum()
    union["all4"] += bits.any(0).sum()
qv = int(quad_visits.sum())
print(f"quadrant visits {qv} (per quadrant {quad_visits.tolist()})")
for k, u in union.items():
    print(f"union {k}: {int(u)} = {u / qv:.3f} of the quadrant visits")
