"""Record the REFERENCE's own call sequence into gstex_cuda (pin the drop-in beyond name
resolution).

Run in the build container only (reads /root/reference, which the GPU box does not have):
    python tests/golden/make_callseq_golden.py
Writes tests/golden/callseq.json (the calls: function, positional / keyword structure, Python scalar types, tensor
dtypes / shapes / contiguity / requires_grad, and which argument is which earlier call's output) and
tests/golden/callseq.npz (the seeded input tensors and the expected outputs).

GStexModel.get_outputs (nerfstudio/models/gstex.py:992-1236) is AST-extracted from the source text and exec'd
UNCHANGED with a stub `self` (the model's parameters: a seeded gstex_amd.scene.make_scene, charts from build_charts),
a stub Cameras object (one sphere_view pose) and a RECORDING gstex_cuda: every call of project_points, get_aabb_2d,
get_num_tiles_hit_2d, spherical_harmonics and texture_gaussians (gstex.py:1077-1080, 1109-1111, 1133-1162) is
recorded and answered by the CPU oracle (oracle/raster.py -- test infrastructure, the checker), so the recorded
downstream arguments (centres, depths, tile counts, SH colours) are the values the reference would pass.  Three
scenarios: "train" (self.training: one 3-channel call, whose backward the replay also checks: the oracle's fp64
gradients for the upstream gradient a photometric loss sends, img / tex / alpha), "eval" (extra_stuff: three
6-channel calls, the third with settings | 1 << 15, gstex.py:1165-1203) and "viewer" (measure_fps: the cached
mapping / fixed-texture path).  The reference's own post-processing of the returned tuples (the 6-tuple unpack at
gstex.py:1172, uv_im / clean_normal_img at :1192-1203) runs on the oracle's outputs here; the GPU replay
(tests/test_gpu_callseq.py) runs the recorded calls through the real gstex_cuda shim.  No reference source is
committed: only the recorded structure, inputs and outputs.
"""
import ast
import json
import math
import os
import sys
import types
from typing import Dict, List, Union

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
REF = "/root/reference/nerfstudio/models/gstex.py"
OUT_JSON = os.path.join(HERE, "callseq.json")
OUT_NPZ = os.path.join(HERE, "callseq.npz")

N_SPLATS, N_TEXELS, H, W, SEED = 300, 4000, 64, 64, 7


def extract(path, names):
    src = open(path).read()
    tree = ast.parse(src)
    found = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name in names and node.name not in found:
            found[node.name] = ast.get_source_segment(src, node)
    assert set(found) == set(names), set(names) - set(found)
    return found


def dedent_method(src):
    lines = src.splitlines()
    ind = len(lines[0]) - len(lines[0].lstrip())
    return "\n".join(ln[ind:] if ln.strip() else ln for ln in lines)


class Recorder:
    """The recording gstex_cuda: each call is logged and answered by the CPU oracle."""

    def __init__(self, scenario):
        from oracle import raster as O

        self.O = O
        self.sc = scenario
        self.calls = []
        self.arrays = {}
        self.produced = {}  # id(tensor) -> (call index, output index)
        self.expect = []  # per call: extra expectations (texture_gaussians: oracle fp64 outputs, margins)
        self._keep = []  # keep recorded outputs alive so their ids stay unique

    def _desc(self, v, key):
        if isinstance(v, torch.Tensor):
            if id(v) in self.produced:
                ci, oi = self.produced[id(v)]
                return {"from": [ci, oi], "requires_grad": bool(v.requires_grad)}
            self.arrays[key] = v.detach().cpu().numpy()
            return {"tensor": key, "dtype": str(v.dtype).replace("torch.", ""), "shape": list(v.shape),
                    "contiguous": bool(v.is_contiguous()), "requires_grad": bool(v.requires_grad)}
        if isinstance(v, (tuple, list)):
            return {"seq": [self._desc(x, f"{key}_{i}") for i, x in enumerate(v)],
                    "type": type(v).__name__}
        if isinstance(v, bool) or v is None:
            return {"py": v, "type": type(v).__name__}
        if isinstance(v, (int, float)):
            return {"py": v, "type": type(v).__name__}
        raise TypeError(f"unrecorded argument type {type(v)}")

    def _record(self, fn, args, kwargs, outs):
        i = len(self.calls)
        base = f"{self.sc}/{i}"
        rec = {"fn": fn, "args": [self._desc(a, f"{base}/a{k}") for k, a in enumerate(args)],
               "kwargs": {k: self._desc(v, f"{base}/k_{k}") for k, v in kwargs.items()}}
        outs_t = outs if isinstance(outs, tuple) else (outs,)
        rec["n_out"] = len(outs_t)
        for k, o in enumerate(outs_t):
            self.arrays[f"{base}/out{k}"] = o.detach().cpu().numpy()
            self.produced[id(o)] = (i, k)
            self._keep.append(o)
        self.calls.append(rec)
        return i

    @staticmethod
    def _cam(viewmat, intr, Hh=0, Ww=0, c2w=None):
        from oracle import raster as O

        fx, fy, cx, cy = intr
        return O.Camera(viewmat.detach().float(), fx, fy, cx, cy, Hh, Ww, 16,
                        None if c2w is None else c2w.detach()[:3, 3].float())

    # --- the gstex_cuda functions gstex.py calls -------------------------------------------------------------
    def project_points(self, means, viewmat, intrinsics):
        xys, depths = self.O.project_points(means.detach(), self._cam(viewmat, intrinsics))
        self._record("project_points", (means, viewmat, intrinsics), {}, (xys, depths))
        return xys, depths

    def get_aabb_2d(self, means, scales, glob_scale, quats, viewmat, intrinsics):
        c, e = self.O.aabb_2d(means, scales, glob_scale, quats, self._cam(viewmat, intrinsics))
        self._record("get_aabb_2d", (means, scales, glob_scale, quats, viewmat, intrinsics), {}, (c, e))
        return c, e

    def get_num_tiles_hit_2d(self, centers, extents, Hh, Ww, block):
        nth = self.O.num_tiles_hit(centers.detach(), extents.detach(), Hh, Ww, block)
        self._record("get_num_tiles_hit_2d", (centers, extents, Hh, Ww, block), {}, nth)
        return nth

    def spherical_harmonics(self, degree, viewdirs, coeffs):
        out = self.O.spherical_harmonics(degree, viewdirs.detach(), coeffs)
        self._record("spherical_harmonics", (degree, viewdirs, coeffs), {}, out)
        return out

    def texture_gaussians(self, *args, **kwargs):
        from helpers import Case, DIFF, oracle_run
        from gstex_amd.scene import View

        (texture_info, texture_dims, centers, extents, depths, nth, rgbs, opacities, means, scales, glob_scale, quats,
         uv0, umap, vmap, texture, viewmat, c2w, fx, fy, cx, cy, Hh, Ww, block, settings) = args
        C = int(texture_info[2])
        cam = self._cam(viewmat, (fx, fy, cx, cy), Hh, Ww, c2w)
        bg = kwargs.get("background")
        d = lambda t: t.detach().clone().float()  # noqa: E731
        inp = self.O.RasterInputs(texture_dims.detach().clone(), d(centers), d(extents), d(depths), d(rgbs),
                                  d(opacities), d(means), d(scales), float(glob_scale), d(quats), d(uv0), d(umap),
                                  d(vmap), d(texture), cam, int(settings), None if bg is None else d(bg))
        view = View(viewmat.detach().float(), c2w.detach().float(), fx, fy, cx, cy, Hh, Ww)
        case = Case(inp, view, C, nth.detach())
        train = self.sc == "train"  # the training call's backward (autograd, engine/trainer.py:460)
        o32, o64, aux, grads = oracle_run(case, grads=train, outputs=("img", "alpha", "tex"))
        names = ("img", "depth", "reg", "alpha", "tex", "normal")
        outs = tuple(o32[k].detach().float() for k in names)
        i = self._record("texture_gaussians", args, kwargs, outs)
        base = f"{self.sc}/{i}"
        for k in names:
            self.arrays[f"{base}/o64_{k}"] = o64[k].detach().double().numpy()
        self.arrays[f"{base}/margin"] = (aux["margin"].detach().numpy() if isinstance(aux["margin"], torch.Tensor)
                                         else np.asarray(aux["margin"]))
        self.calls[i]["train_grads"] = bool(train)
        if train:
            _, _, _, g32 = oracle_run(case, grads=True, grad_dtype=torch.float32, outputs=("img", "alpha", "tex"))
            self.arrays[f"{base}/flip_mask"] = case.flip_mask.numpy()
            for k in DIFF:
                self.arrays[f"{base}/g64_{k}"] = grads[k].double().numpy()
                self.arrays[f"{base}/g32_{k}"] = g32[k].double().numpy()
        # ordinary tensors with autograd history, as the reference's caller expects (it only slices / unpacks)
        return outs


class Cameras:  # isinstance target of get_outputs' assert (nerfstudio.cameras.cameras.Cameras)
    def __init__(self, view):
        self.camera_to_worlds = view.c2w_gl[None, :3, :].clone()
        self.fx = torch.tensor([[view.fx]])
        self.fy = torch.tensor([[view.fy]])
        self.cx = torch.tensor([[view.cx]])
        self.cy = torch.tensor([[view.cy]])
        self.width = torch.tensor([[view.W]])
        self.height = torch.tensor([[view.H]])
        self.shape = (1,)

    def rescale_output_resolution(self, s):
        assert s == 1


class Config:
    background_color = "random"
    sh_degree = 3
    sh_degree_interval = 1000
    fix_init = False
    use_normal_loss = False


class JaggedStub:
    def __init__(self, t):
        self.t = t
        self.total_size = t.shape[0]

    def get_texture(self):
        return self.t


def make_self(scenario, fns):
    from gstex_amd.scene import make_scene

    sc = make_scene(N_SPLATS, N_TEXELS, seed=SEED)
    s = types.SimpleNamespace()
    P = lambda t: torch.nn.Parameter(t.detach().clone())  # noqa: E731
    s.means, s.scales, s.quats, s.opacities = P(sc.means), P(sc.log_scales), P(sc.quats), P(sc.opacity_logits)
    s.features_dc, s.features_rest = P(sc.features_dc), P(sc.features_rest)
    s.mappings = sc.mappings.clone()
    s.texture_dims = sc.texture_dims.clone()
    s.texture_dc = JaggedStub(P((sc.texture - 0.5) / 0.28209479177387814))
    s.num_points = sc.n
    s.settings = (1 << 9) | (1 << 10)
    s.config = Config()
    s.device = torch.device("cpu")
    s.step = 3000
    s.training = scenario == "train"
    s.measure_fps = scenario == "viewer"
    s.mapping_set = False
    s.texture_set = False
    s.edit_texture = None
    s.test_colors = torch.rand((sc.n, 3), generator=torch.Generator().manual_seed(SEED + 1))
    s.background_color = torch.tensor([1.0, 1.0, 1.0])
    s.load_draw_camera = lambda camera: None
    s._get_downscale_factor = lambda: 1
    s.get_uv_mapping = types.MethodType(fns["get_uv_mapping"], s)
    return s


def main():
    from gstex_amd.scene import sphere_view
    from gstex_cuda._torch_impl import quat_to_rotmat

    src = {k: v for k, v in extract(REF, ["get_outputs", "get_uv_mapping", "SH2RGB", "projection_matrix",
                                          "depths_to_points", "depth_to_normal"]).items()}
    view = sphere_view(2, H, W)
    # the reference derives viewmat / c2w from the OpenGL camera_to_worlds (gstex.py:1031-1042): undo the y/z flip
    c2w_cv = view.c2w.double()
    view.c2w_gl = (c2w_cv @ torch.diag(torch.tensor([1.0, -1.0, -1.0, 1.0], dtype=torch.float64))).float()
    meta, arrays = {"source": "nerfstudio/models/gstex.py:992-1236 GStexModel.get_outputs (AST-extracted, run "
                              "unchanged with a stub self / camera and a recording gstex_cuda)",
                    "n_splats": N_SPLATS, "n_texels": N_TEXELS, "H": H, "W": W, "seed": SEED, "scenarios": {}}, {}
    for scenario in ("train", "eval", "viewer"):
        rec = Recorder(scenario)
        ns = dict(torch=torch, math=math, np=np, Dict=Dict, Union=Union, List=List, Cameras=Cameras,
                  renderers=types.SimpleNamespace(BACKGROUND_COLOR_OVERRIDE=None), quat_to_rotmat=quat_to_rotmat,
                  project_points=rec.project_points, get_aabb_2d=rec.get_aabb_2d,
                  get_num_tiles_hit_2d=rec.get_num_tiles_hit_2d, spherical_harmonics=rec.spherical_harmonics,
                  texture_gaussians=rec.texture_gaussians)
        fns = {}
        for name in ("SH2RGB", "projection_matrix", "depths_to_points", "depth_to_normal", "get_uv_mapping",
                     "get_outputs"):
            code = "from __future__ import annotations\n" + dedent_method(src[name])
            exec(compile(code, f"<gstex.py:{name}>", "exec"), ns)
            fns[name] = ns[name]
        self_ = make_self(scenario, fns)
        torch.manual_seed(SEED)  # the random training background (gstex.py:1014)
        images = fns["get_outputs"](self_, Cameras(view))
        meta["scenarios"][scenario] = {"calls": rec.calls, "image_keys": sorted(images)}
        arrays.update(rec.arrays)
        for k, v in images.items():
            if isinstance(v, torch.Tensor):
                arrays[f"{scenario}/images/{k}"] = v.detach().cpu().numpy()
        print(scenario, [c["fn"] for c in rec.calls], sorted(images))
    json.dump(meta, open(OUT_JSON, "w"), indent=1)
    np.savez_compressed(OUT_NPZ, **arrays)
    print("wrote", OUT_JSON, OUT_NPZ, sum(a.nbytes for a in arrays.values()) / 1e6, "MB raw")


if __name__ == "__main__":
    main()
