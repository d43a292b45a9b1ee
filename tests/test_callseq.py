"""The reference's own call sequence into gstex_cuda, as recorded from nerfstudio/models/gstex.py:992-1236
(tests/golden/make_callseq_golden.py), checked against the drop-in surface without a GPU: the recorded structure
(what the reference passes) and that every recorded call binds to the shim's signature as the reference makes it.
The GPU replay through the HIP library is tests/test_gpu_callseq.py."""
import inspect

import numpy as np
import pytest

from callseq import IMPORTS, load, resolve

EXPECTED = {
    "train": ["project_points", "get_aabb_2d", "get_num_tiles_hit_2d", "spherical_harmonics", "texture_gaussians"],
    "eval": ["project_points", "get_aabb_2d", "get_num_tiles_hit_2d", "spherical_harmonics", "texture_gaussians",
             "texture_gaussians", "texture_gaussians"],
    "viewer": ["project_points", "get_aabb_2d", "get_num_tiles_hit_2d", "spherical_harmonics", "texture_gaussians"],
}


@pytest.fixture(scope="module")
def golden():
    return load()


def test_recorded_sequence_and_argument_structure(golden):
    meta, arrays = golden
    n = meta["n_splats"]
    for sc, fns in EXPECTED.items():
        calls = meta["scenarios"][sc]["calls"]
        assert [c["fn"] for c in calls] == fns, sc
        for c in calls:
            if c["fn"] in ("project_points", "get_aabb_2d"):
                vm = c["args"][1 if c["fn"] == "project_points" else 4]
                assert vm["shape"] == [3, 4]  # viewmat.squeeze()[:3, :] (gstex.py:1077, 1079)
                intr = c["args"][-1]
                assert intr["type"] == "tuple" and all(d["type"] == "float" for d in intr["seq"])
            if c["fn"] == "get_aabb_2d":
                assert c["args"][2] == {"py": 1, "type": "int"}  # glob_scale: the int literal 1
            if c["fn"] != "texture_gaussians":
                continue
            a, kw = c["args"], c["kwargs"]
            assert len(a) == 26 and set(kw) == {"background", "use_torch_impl"}
            info = a[0]
            assert info["type"] == "tuple" and [d["type"] for d in info["seq"]] == ["int"] * 3
            assert info["seq"][0]["py"] == n and info["seq"][1]["py"] == 1
            assert info["seq"][2]["py"] == (6 if sc == "eval" else 3)  # texture_channels (gstex.py:1085-1087)
            assert a[10] == {"py": 1, "type": "int"}  # glob_scale
            assert a[16]["shape"] == [3, 4] and a[17]["shape"] == [4, 4]
            assert a[17]["contiguous"] is False  # c2w = viewmat.squeeze().inverse() (gstex.py:1043)
            assert [d["type"] for d in a[18:22]] == ["float"] * 4 and [d["type"] for d in a[22:26]] == ["int"] * 4
            assert kw["use_torch_impl"] == {"py": False, "type": "bool"}
            assert np.all(arrays[kw["background"]["tensor"]] == 0.0)  # background=torch.zeros_like(background)
            # centres / extents / depths / tile counts / colours are the outputs of the calls before it
            assert [a[k]["from"] for k in (2, 3, 4, 5)] == [[1, 0], [1, 1], [0, 1], [2, 0]]
            # colours: the SH output for the image render, the fixed test colours for eval's two extra renders
            assert a[6].get("from") == ([3, 0] if c is calls[4] else None)
        settings = [c["args"][25]["py"] for c in calls if c["fn"] == "texture_gaussians"]
        if sc == "eval":
            assert settings == [1536, 1536, 1536 | (1 << 15)]  # the third call: the clean-normal render (gstex.py:1198)
        else:
            assert settings == [1536]


def test_recorded_calls_bind_to_the_shim_signatures(golden):
    """Each recorded call, with its positional / keyword structure, binds to the gstex_cuda function the reference
    imports (gstex.py:29-32) -- the same names, arity and keywords (no GPU needed)."""
    meta, _ = golden
    for sc in EXPECTED:
        for c in meta["scenarios"][sc]["calls"]:
            fn = resolve(c["fn"])
            sig = inspect.signature(fn)
            sig.bind(*[object()] * len(c["args"]), **{k: object() for k in c["kwargs"]})
    assert set(IMPORTS) == {c["fn"] for s in meta["scenarios"].values() for c in s["calls"]}


def test_reference_postprocessing_images_recorded(golden):
    """The reference's own handling of the returned tuples (the 6-tuple unpack at gstex.py:1172 and the eval images
    of gstex.py:1183-1236) ran on the oracle's outputs when the fixture was made: the images it returned are there
    for the GPU replay to compare with."""
    meta, arrays = golden
    assert set(meta["scenarios"]["train"]["image_keys"]) >= {"rgb", "depth", "accumulation", "normal_im", "reg"}
    assert set(meta["scenarios"]["eval"]["image_keys"]) >= {"rgb", "test", "edit", "clean_normal_img", "uv"}
    assert meta["scenarios"]["viewer"]["image_keys"] == ["background", "rgb"]
    for sc in EXPECTED:
        rgb = arrays[f"{sc}/images/rgb"]
        assert rgb.shape == (meta["H"], meta["W"], 3) and rgb.min() >= 0.0 and rgb.max() <= 1.0
