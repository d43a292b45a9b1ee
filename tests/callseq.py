"""Loader / replayer of the reference's recorded gstex_cuda call sequence (tests/golden/callseq.{json,npz}, made by
tests/golden/make_callseq_golden.py from nerfstudio/models/gstex.py:992-1236 GStexModel.get_outputs)."""
from __future__ import annotations

import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

# where the reference imports each function from (gstex.py:29-32): the replay resolves them the same way
IMPORTS = {
    "project_points": ("gstex_cuda.get_aabb_2d", "project_points"),
    "get_aabb_2d": ("gstex_cuda.get_aabb_2d", "get_aabb_2d"),
    "get_num_tiles_hit_2d": ("gstex_cuda.get_aabb_2d", "get_num_tiles_hit_2d"),
    "spherical_harmonics": ("gstex_cuda.sh", "spherical_harmonics"),
    "texture_gaussians": ("gstex_cuda.texture", "texture_gaussians"),
}


def load():
    meta = json.load(open(os.path.join(GOLDEN, "callseq.json")))
    arrays = dict(np.load(os.path.join(GOLDEN, "callseq.npz")))
    return meta, arrays


def resolve(fn: str):
    import importlib

    mod, name = IMPORTS[fn]
    return getattr(importlib.import_module(mod), name)


def build(desc, arrays, outs, device, leaves=None, grads=False):
    """A recorded argument back to its value: a tensor from the npz (on `device`, with the recorded strides'
    contiguity), an earlier call's replayed output ("from"), or the Python value with its recorded type."""
    if "from" in desc:
        ci, oi = desc["from"]
        v = outs[ci][oi]
        if grads and desc["requires_grad"]:
            v = v.detach().clone().requires_grad_(True)  # a leaf at the raster boundary (the gradient check)
            if leaves is not None:
                leaves.append((desc, v))
        return v
    if "tensor" in desc:
        t = torch.from_numpy(np.ascontiguousarray(arrays[desc["tensor"]])).to(device)
        if not desc["contiguous"]:
            t = t.t().contiguous().t()  # the recorded argument was not contiguous (c2w = viewmat.inverse())
            assert not t.is_contiguous() or t.dim() < 2
        if grads and desc["requires_grad"]:
            t.requires_grad_(True)
            if leaves is not None:
                leaves.append((desc, t))
        return t
    if "seq" in desc:
        vals = [build(d, arrays, outs, device, leaves, grads) for d in desc["seq"]]
        return tuple(vals) if desc["type"] == "tuple" else vals
    t = desc["type"]
    v = desc["py"]
    return {"int": int, "float": float, "bool": bool, "NoneType": lambda x: None}[t](v)


def expected_outputs(scenario: str, i: int, n_out: int, arrays):
    return [torch.from_numpy(arrays[f"{scenario}/{i}/out{k}"]) for k in range(n_out)]
