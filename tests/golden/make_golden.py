"""Generate host-side golden vectors from the REFERENCE's own pure-torch functions.

Run in the build container only (it reads /root/reference, which does not exist on the GPU box):
    python tests/golden/make_golden.py
The reference module cannot be imported whole (gstex_cuda, tyro, plyfile, open3d, cv2, ... are
absent), so the individual functions are AST-extracted from the source text and exec'd with the
minimum of stubs; only their inputs/outputs are committed (tests/golden/host_goldens.npz).

Functions exercised (file:line):
  models/jagged_texture.py:10  texture_dims_to_int_coords
  models/jagged_texture.py:23  texture_dims_to_query
  models/gstex.py:68           random_quat_tensor
  models/gstex.py:86,94        RGB2SH, SH2RGB
  models/gstex.py:841          GStexModel.build_charts   (self stubbed)
  models/gstex.py:975          GStexModel.get_uv_mapping (quat_to_rotmat := rotations.quaternion_to_matrix)
"""
import ast
import math
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference/nerfstudio"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "host_goldens.npz")


def extract(path, names):
    src = open(path).read()
    tree = ast.parse(src)
    found = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name in names and node.name not in found:
            found[node.name] = ast.get_source_segment(src, node)
    missing = set(names) - set(found)
    assert not missing, missing
    return found


def main():
    sys.path.insert(0, "/root/reference")
    from nerfstudio.utils.rotations import quaternion_to_matrix  # pure torch, importable

    ns = {"torch": torch, "np": np, "math": math, "quat_to_rotmat": quaternion_to_matrix}
    jt = extract(f"{REF}/models/jagged_texture.py", ["texture_dims_to_int_coords", "texture_dims_to_query"])
    gs = extract(f"{REF}/models/gstex.py", ["random_quat_tensor", "RGB2SH", "SH2RGB", "build_charts",
                                             "get_uv_mapping"])
    for code in list(jt.values()) + list(gs.values()):
        exec(code, ns)

    out = {}
    torch.manual_seed(42)
    q = ns["random_quat_tensor"](64)
    out["rq_seed"] = np.array([42])
    out["rq_out"] = q.numpy()

    rgb = torch.rand(32, 3)
    out["rgb_in"] = rgb.numpy()
    out["rgb2sh_out"] = ns["RGB2SH"](rgb).numpy()
    out["sh2rgb_out"] = ns["SH2RGB"](rgb).numpy()

    # build_charts on seeded log-uniform scales (as SURVEY §8 measured)
    g = torch.Generator().manual_seed(7)
    for tag, n, pix in (("a", 2000, 5e4), ("b", 500, 1e4), ("c", 3000, 2e5)):
        log_scales = torch.log(10 ** (-2.5 + 1.5 * torch.rand((n, 3), generator=g)))
        fake = types.SimpleNamespace()
        fake.config = types.SimpleNamespace(pixel_num=pix, sigma_factor=3.0)
        fake.scales = log_scales
        fake.mappings = torch.ones((n, 2))
        fake.texture_dims = torch.ones((n, 3), dtype=torch.int32)
        fake.pixel_scale = 10.0 * torch.ones(1)
        fake.num_points = n
        fake.texture_dc = types.SimpleNamespace(init_from_dims=lambda dims: None)
        fake.update_edit_texture = lambda: None
        fake.edit_texture = None
        ns["build_charts"](fake)
        out[f"bc_{tag}_log_scales"] = log_scales.numpy()
        out[f"bc_{tag}_pixel_num"] = np.array([pix])
        out[f"bc_{tag}_dims"] = fake.texture_dims.numpy()
        out[f"bc_{tag}_mappings"] = fake.mappings.numpy()
        out[f"bc_{tag}_pixel_scale"] = fake.pixel_scale.numpy()
        if tag == "b":
            ids, iuv = ns["texture_dims_to_int_coords"](fake.texture_dims)
            qids, quv = ns["texture_dims_to_query"](fake.texture_dims)
            out["tq_dims"] = fake.texture_dims.numpy()
            out["tq_int_ids"] = ids.numpy()
            out["tq_int_uv"] = iuv.numpy()
            out["tq_ids"] = qids.numpy()
            out["tq_uv"] = quv.numpy()

    # get_uv_mapping (self unused beyond the call)
    quats = torch.randn(128, 4, generator=g)
    quats = quats / quats.norm(dim=-1, keepdim=True)
    mappings = torch.rand(128, 2, generator=g) + 0.1
    means = torch.randn(128, 3, generator=g)
    uv0, umap, vmap = ns["get_uv_mapping"](None, means, quats, mappings)
    out["uvm_quats"] = quats.numpy()
    out["uvm_mappings"] = mappings.numpy()
    out["uvm_uv0"] = uv0.numpy()
    out["uvm_umap"] = umap.numpy()
    out["uvm_vmap"] = vmap.numpy()

    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
