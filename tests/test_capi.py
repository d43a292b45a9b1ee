"""C-ABI boundary checks that need no GPU: the library loads, exports every symbol include/gstex_hip.h
declares, and rejects invalid arguments (before any HIP call) with a status and a message."""
import ctypes
import os
import re

import pytest

from gstex_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gstex_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gstex_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build()
    return _lib.load()


def test_every_header_symbol_is_exported_and_bound(lib):
    syms = declared_symbols()
    assert len(syms) >= 29
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in gstex_hip.h but not exported"
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature in gstex_amd/_lib.py"
    assert set(_lib.SIGNATURES) == set(syms), "ctypes signatures out of sync with the header"


def test_abi_version(lib):
    assert lib.gstex_abi_version() == _lib.ABI_VERSION == 18


def test_workspace_size_queries(lib):
    assert lib.gstex_scan_workspace_size(0) >= 4
    small = lib.gstex_bin_workspace_size(100, 1000, 64)
    big = lib.gstex_bin_workspace_size(100, 100000, 64)
    assert big > small > 0
    # keys (8 B) + scratch (8 B) + rank (4 B) per intersection dominate
    assert big - small >= 20 * (100000 - 1000) - 3 * 256


def _cam(H=32, W=32, block=16):
    return _lib.GstexCamera(None, None, 100.0, 100.0, 16.0, 16.0, H, W, block)


def _status(lib, name, *args):
    rc = getattr(lib, name)(*args)
    return rc, _lib.last_error()


def test_bin_sort_rejects_non16_block(lib):
    rc, msg = _status(lib, "gstex_bin_sort", 10, 10, None, None, None, None, None, 32, 32, 8, None, None, None, None,
                      0, None)
    assert rc == 1 and "block_width must be 16" in msg


def test_raster_rejects_bad_channels_and_settings(lib):
    cam = _cam()
    rc, msg = _status(lib, "gstex_raster_fwd", ctypes.byref(cam), 9, 0, None, None, None, None, None, None, None, 0, 1.0,
                      0.0, None, None, None, None, None, None, None, 0, None, None)
    assert rc == 1 and "channels" in msg
    rc, msg = _status(lib, "gstex_raster_fwd", ctypes.byref(cam), 3, 1 << 2, None, None, None, None, None, None, None, 0,
                      1.0, 0.0, None, None, None, None, None, None, None, 0, None, None)
    assert rc == 3 and "unsupported settings" in msg
    bad = _cam(block=8)
    rc, msg = _status(lib, "gstex_raster_bwd", ctypes.byref(bad), 3, 0, None, None, None, None, None, None, None, 0,
                      1.0, 0.0, None, None, None, None, None, None, None, 0, None, None, None, None, None)
    assert rc == 1 and "block_width" in msg


def test_raster_aux_bytes(lib):
    # cull-bit words (ceil(I / 64) + n_tiles + 1) * 4 x 8 B, then per backward unit (4 per slot; ceil(I / 256) +
    # n_tiles + 1 slots) cost + order (4 B each), the order's scratch, slot tiles
    # (4 B per slot) and a checkpoint of (4 + C + 6) fields x 64 lanes per unit, each array 256-B aligned
    def al(x):
        return (x + 255) // 256 * 256

    for n_isect, n_tiles, c in [(0, 1, 3), (1_915_389, 2500, 3), (12345, 77, 6)]:
        slots = (n_isect + 255) // 256 + n_tiles + 1
        expect = (al(((n_isect + 63) // 64 + n_tiles + 1) * 32) + 2 * al(slots * 16) + al(lib.gstex_unit_order_scratch_words() * 4) + al(slots * 4)
                  + al(slots * 4 * (4 + c + 6) * 64 * 4))
        assert lib.gstex_raster_aux_bytes(n_isect, n_tiles, c) == expect
    assert lib.gstex_raster_aux_bytes(-1, 1, 3) == 0 and lib.gstex_raster_aux_bytes(1, 1, 9) == 0


def test_sh_rejects_degree(lib):
    rc, msg = _status(lib, "gstex_sh_fwd", 4, 5, 36, None, None, None, None)
    assert rc == 1 and "degree" in msg
    rc, msg = _status(lib, "gstex_sh_fwd", 4, 3, 9, None, None, None, None)
    assert rc == 1 and "coefficients" in msg


def test_empty_inputs_are_noops(lib):
    cam = _cam()
    # n == 0 returns before touching the device
    assert lib.gstex_project_points(0, None, ctypes.byref(cam), None, None, None) == 0
    assert lib.gstex_aabb_2d(0, None, None, 1.0, None, ctypes.byref(cam), None, None, None) == 0
    assert lib.gstex_num_tiles_hit(0, None, None, 32, 32, 16, None, None) == 0
    assert lib.gstex_sh_fwd(0, 3, 16, None, None, None, None) == 0
    assert lib.gstex_texture_sample(0, 3, None, None, 0, None, None, None) == 0


def test_null_pointer_is_an_error(lib):
    cam = _cam()
    rc, msg = _status(lib, "gstex_project_points", 5, None, ctypes.byref(cam), None, None, None)
    assert rc == 1 and "null" in msg


def test_python_wrappers_refuse_cpu_tensors():
    import torch

    from gstex_amd import ops

    with pytest.raises(RuntimeError, match="HIP"):
        ops.project_points(torch.zeros(4, 3), torch.eye(4)[:3], (1.0, 1.0, 0.0, 0.0))


def test_adam_rejects_bad_tables(lib):
    from gstex_amd import _lib

    rc, msg = _status(lib, "gstex_adam_step", 17, None, 0.9, 0.999, 1e-15, None)
    assert rc == 1 and "n_tensors" in msg
    t = (_lib.GstexAdamTensor * 1)(_lib.GstexAdamTensor(None, None, None, None, 10, 1e-3, 1.0))
    rc, msg = _status(lib, "gstex_adam_step", 1, t, 0.9, 0.999, 1e-15, None)
    assert rc == 1 and "null pointer" in msg
    t = (_lib.GstexAdamTensor * 1)(_lib.GstexAdamTensor(None, None, None, None, 0, 1e-3, 1.0))
    assert _status(lib, "gstex_adam_step", 1, t, 0.9, 0.999, 1e-15, None)[0] == 0  # empty: no launch


def test_loss_rejects_small_images_and_channels(lib):
    assert lib.gstex_loss_workspace_size(10, 64) == 0
    assert lib.gstex_loss_workspace_size(64, 64) > 9 * 54 * 54 * 4
    win = (ctypes.c_float * 11)()
    rc, msg = _status(lib, "gstex_loss_fwd", 8, 64, 3, None, None, None, None, None, win, 0.2, None, None, None, 0,
                      None)
    assert rc == 1 and "window" in msg
    rc, msg = _status(lib, "gstex_loss_bwd", 64, 64, 2, None, None, None, None, None, win, 0.2, None, None, None,
                      None, None, 0, None)
    assert rc == 1 and "channels" in msg


def test_activate_and_sh_rest_reject_bad_args(lib):
    rc, msg = _status(lib, "gstex_activate_fwd", 10, None, None, None, None, None, 1, None, None, None, None, None,
                      None, None, None, None)
    assert rc == 1 and "mappings_stride" in msg
    rc, msg = _status(lib, "gstex_activate_fwd", 10, None, None, None, None, None, 2, None, None, None, None, None,
                      None, None, None, None)
    assert rc == 1 and "null pointer" in msg
    rc, msg = _status(lib, "gstex_sh_rest_fwd", 4, 5, 35, None, None, None, None)
    assert rc == 1 and "degree" in msg
    rc, msg = _status(lib, "gstex_sh_rest_fwd", 4, 3, 14, None, None, None, None)
    assert rc == 1 and "coefficients" in msg
    assert lib.gstex_activate_fwd(0, None, None, None, None, None, 2, None, None, None, None, None, None, None, None,
                                  None) == 0


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors in gstex_amd/_lib.py have the header's sizes and field offsets (gcc on the header)."""
    import subprocess

    structs = {"gstex_camera": _lib.GstexCamera, "gstex_pair_guard": _lib.GstexPairGuard,
               "gstex_adam_tensor": _lib.GstexAdamTensor,
               "gstex_train_prologue_args": _lib.GstexTrainPrologueArgs,
               "gstex_train_epilogue_args": _lib.GstexTrainEpilogueArgs}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "gstex_hip.h"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f in cls._fields_:
            lines.append(f'printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], check=True, capture_output=True,
                                                        text=True).stdout.splitlines())
    for cname, cls in structs.items():
        assert int(got[f"{cname} size"]) == ctypes.sizeof(cls), cname
        for f in cls._fields_:
            assert int(got[f"{cname} {f[0]}"]) == getattr(cls, f[0]).offset, f"{cname}.{f[0]}"


def test_train_prologue_scan_bytes(lib):
    for n in (0, 1, 127, 128, 1025, 200_000):
        b = lib.gstex_train_prologue_scan_bytes(n)
        assert b >= lib.gstex_scan_workspace_size(n) and b >= 4 * ((n + 255) // 256)  # one word per 256-splat block


def test_train_prologue_rejects_null_args(lib):
    rc, msg = _status(lib, "gstex_train_prologue", None, None)
    assert rc != 0 and "null" in msg
    rc, msg = _status(lib, "gstex_train_epilogue", None, None)
    assert rc != 0 and "invalid" in msg
