"""ctypes binding of libgstex_hip.so (the C-ABI declared in include/gstex_hip.h).

The shared library is built in-tree (``make -C gstex_amd/csrc`` or ``__graft_entry__.build()``).
There is no fallback: if the library is missing every op raises, so a GPU run can never silently
fall back to a CPU path.  ``torch`` must be imported before the library is loaded so that the HIP
runtime torch ships (soname libamdhip64.so.7) is the one the library binds to.
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import POINTER, c_char_p, c_double, c_float, c_int32, c_int64, c_size_t, c_void_p

import torch  # noqa: F401  (load torch's HIP runtime first)

LIB_PATH = os.environ.get("GSTEX_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgstex_hip.so")

ABI_VERSION = 18
REC_FLOATS = 32
HP_DOUBLES = 12  # GSTEX_HP_DOUBLES: the fp64 row of a near-edge-on splat (gstex_raster_setup hp_records)
PARTIAL_FLOATS = 32  # GSTEX_PARTIAL_FLOATS: floats between partial rows of a backward with geometry gradients
PARTIAL_FLOATS_PHOTO = 24  # GSTEX_PARTIAL_FLOATS_PHOTO: ... without (the photometric training step)
SETTING_AA_BLUR = 1 << 9
SETTING_DIST_REG = 1 << 10
SETTING_EDIT = 1 << 13
SETTING_EVAL_NORMAL = 1 << 15
SETTING_AUX_ZEROED = 1 << 28  # GSTEX_SETTING_AUX_ZEROED: the prologue zeroed the forward's accumulated aux span


class GstexCamera(ctypes.Structure):
    _fields_ = [
        ("viewmat", c_void_p),
        ("c2w", c_void_p),
        ("fx", c_float),
        ("fy", c_float),
        ("cx", c_float),
        ("cy", c_float),
        ("H", c_int32),
        ("W", c_int32),
        ("block", c_int32),
    ]


class GstexAdamTensor(ctypes.Structure):
    _fields_ = [
        ("param", c_void_p),
        ("grad", c_void_p),
        ("exp_avg", c_void_p),
        ("exp_avg_sq", c_void_p),
        ("numel", c_int64),
        ("step_size", c_float),
        ("bias_correction2_sqrt", c_float),
    ]


class GstexPairGuard(ctypes.Structure):
    _fields_ = [
        ("capacity", c_int64),
        ("step_flag", c_void_p),
        ("host_count", c_void_p),
        ("first", c_int32),
    ]


ADAM_MAX_TENSORS = 16


class GstexTrainPrologueArgs(ctypes.Structure):
    """gstex_train_prologue_args (ABI 17): the launches of a training render before its raster forward."""
    _fields_ = [("n", c_int32), ("sh_degree", c_int32), ("n_rest", c_int32), ("map_cols", c_int32),
                ("capacity", c_int64), ("cam", GstexCamera), ("guard", GstexPairGuard)] + [
        (name, c_void_p) for name in (
            "means", "quats", "log_scales", "opac_logits", "mappings", "campos", "features_rest", "texture_dims",
            "quats_n", "scales", "opacities", "uv0", "umap", "vmap", "viewdirs", "depths", "centers", "extents",
            "num_tiles_hit", "rgbs", "offsets", "scan_workspace")] + [("scan_workspace_bytes", c_size_t)] + [
        (name, c_void_p) for name in (
            "records", "tile_ranges", "sorted_ids", "sorted_slots", "tile_order", "bin_workspace")] + [
        ("bin_workspace_bytes", c_size_t), ("raster_aux", c_void_p), ("raster_aux_bytes", c_size_t),
        ("raster_channels", c_int32), ("hp_records", c_void_p)]


class GstexTrainEpilogueArgs(ctypes.Structure):
    """gstex_train_epilogue_args (ABI 17): the training render's backward after the raster backward."""
    _fields_ = [("n", c_int32), ("sh_degree", c_int32), ("n_rest", c_int32), ("cam", GstexCamera)] + [
        (name, c_void_p) for name in (
            "means", "scales", "quats_n", "quats", "log_scales", "opacities", "umap", "vmap", "viewdirs",
            "num_tiles_hit", "offsets", "partials", "v_means", "v_quats", "v_log_scales", "v_opac_logits",
            "v_features_rest", "v_scales_act", "v_quats_n", "v_rgbs", "v_opacities_act", "v_centers", "v_uv0")]


ADAM_ZERO_GRAD = 1  # GSTEX_ADAM_ZERO_GRAD
ADAM_GRID_SHIFT = 8  # GSTEX_ADAM_GRID_SHIFT
_P = c_void_p
_CAM = POINTER(GstexCamera)

# name -> (restype, argtypes); must mirror include/gstex_hip.h
SIGNATURES = {
    "gstex_last_error": (c_char_p, []),
    "gstex_abi_version": (c_int32, []),
    "gstex_project_points": (c_int32, [c_int32, _P, _CAM, _P, _P, _P]),
    "gstex_project_points_bwd": (c_int32, [c_int32, _P, _CAM, _P, _P, _P, _P]),
    "gstex_aabb_2d": (c_int32, [c_int32, _P, _P, c_float, _P, _CAM, _P, _P, _P]),
    "gstex_aabb_2d_bwd": (c_int32, [c_int32, _P, _P, c_float, _P, _CAM, _P, _P, _P, _P, _P]),
    "gstex_num_tiles_hit": (c_int32, [c_int32, _P, _P, c_int32, c_int32, c_int32, _P, _P]),
    "gstex_preprocess": (c_int32, [c_int32, _P, _P, c_float, _P, _CAM, _P, _P, _P, _P, _P]),
    "gstex_scan_workspace_size": (c_size_t, [c_int32]),
    "gstex_scan_offsets": (c_int32, [c_int32, _P, _P, _P, c_size_t, _P]),
    "gstex_bin_workspace_size": (c_size_t, [c_int32, c_int64, c_int32]),
    "gstex_bin_sort": (
        c_int32,
        [c_int32, c_int64, _P, _P, _P, _P, _P, c_int32, c_int32, c_int32, _P, _P, _P, _P, c_size_t, _P],
    ),
    "gstex_bin_sort_ordered": (
        c_int32,
        [c_int32, c_int64, _P, _P, _P, _P, _P, c_int32, c_int32, c_int32, _P, _P, _P, _P, _P, c_size_t, _P],
    ),
    "gstex_tile_order": (c_int32, [c_int32, _P, _P, _P]),
    "gstex_scan_offsets_guarded": (c_int32, [c_int32, _P, _P, _P, c_size_t, POINTER(GstexPairGuard), _P]),
    "gstex_bin_sort_capped": (
        c_int32,
        [c_int32, c_int64, _P, _P, _P, _P, _P, c_int32, c_int32, c_int32, _P, _P, _P, _P, _P, c_size_t, _P],
    ),
    "gstex_host_words_alloc": (c_int32, [c_int32, POINTER(c_void_p), POINTER(c_void_p)]),
    "gstex_host_words_free": (c_int32, [c_void_p]),
    "gstex_event_create": (c_int32, [c_int32, POINTER(c_void_p)]),
    "gstex_event_record": (c_int32, [c_void_p, c_void_p]),
    "gstex_event_elapsed": (c_int32, [c_void_p, c_void_p, POINTER(ctypes.c_float)]),
    "gstex_stream_wait_event": (c_int32, [c_void_p, c_void_p]),
    "gstex_event_destroy": (c_int32, [c_void_p]),
    "gstex_raster_setup": (
        c_int32,
        [c_int32, _P, _P, c_float, _P, _P, _P, _P, _P, _P, _P, _P, _P, _CAM, _P, _P, _P],
    ),
    "gstex_raster_fwd": (
        c_int32,
        [_CAM, c_int32, c_int32, _P, _P, _P, _P, _P, _P, _P, c_int64, c_float, c_float, _P, _P, _P, _P, _P, _P, _P,
         c_int64, _P, _P],
    ),
    "gstex_raster_fwd_zero": (
        c_int32,
        [_CAM, c_int32, c_int32, _P, _P, _P, _P, _P, _P, _P, c_int64, c_float, c_float, _P, _P, _P, _P, _P, _P, _P,
         c_int64, _P, _P, c_int64, _P, c_int64, _P],
    ),
    "gstex_raster_aux_bytes": (c_size_t, [c_int64, c_int32, c_int32]),
    "gstex_unit_order": (c_int32, [c_int32, _P, _P, _P, _P]),
    "gstex_unit_order_scratch_words": (c_size_t, []),
    "gstex_raster_bwd": (
        c_int32,
        [_CAM, c_int32, c_int32, _P, _P, _P, _P, _P, _P, _P, c_int64, c_float, c_float, _P, _P, _P, _P, _P, _P, _P,
         c_int64, _P, _P, _P, _P, _P],
    ),
    "gstex_raster_bwd_zero": (
        c_int32,
        [_CAM, c_int32, c_int32, _P, _P, _P, _P, _P, _P, _P, c_int64, c_float, c_float, _P, _P, _P, _P, _P, _P, _P,
         c_int64, _P, _P, _P, _P, _P, c_int64, _P],
    ),
    "gstex_raster_setup_bwd": (
        c_int32,
        [c_int32, _P, _P, c_float, _P, _P, _P, _P, _P, _P, _P, _P, c_int32, c_int64, _CAM, _P, _P, _P, _P, _P, _P, _P,
         _P],
    ),
    "gstex_raster_setup_bwd_aabb": (
        c_int32,
        [c_int32, _P, _P, c_float, _P, _P, _P, _P, _P, _P, _P, _P, c_int32, c_int64, _CAM, _P, _P, _P, _P, _P, _P, _P,
         _P],
    ),
    "gstex_sh_fwd": (c_int32, [c_int32, c_int32, c_int32, _P, _P, _P, _P]),
    "gstex_sh_bwd": (c_int32, [c_int32, c_int32, c_int32, _P, _P, _P, _P]),
    "gstex_texture_sample": (c_int32, [c_int64, c_int32, _P, _P, c_int64, _P, _P, _P]),
    "gstex_texture_sample_bwd": (c_int32, [c_int64, c_int32, _P, c_int64, _P, _P, _P, _P]),
    "gstex_activate_fwd": (c_int32, [c_int32, _P, _P, _P, _P, _P, c_int32, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "gstex_activate_bwd": (c_int32, [c_int32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "gstex_sh_rest_fwd": (c_int32, [c_int32, c_int32, c_int32, _P, _P, _P, _P]),
    "gstex_sh_rest_bwd": (c_int32, [c_int32, c_int32, c_int32, _P, _P, _P, _P]),
    "gstex_texture_edit": (c_int32, [_CAM, c_int32, _P, _P, _P, _P, _P, _P, _P, _P, c_int64, _P, _P]),
    "gstex_loss_workspace_size": (c_size_t, [c_int32, c_int32]),
    "gstex_loss_fwd": (c_int32, [c_int32, c_int32, c_int32, _P, _P, _P, _P, _P, POINTER(c_float), c_float, _P, _P,
                                 _P, c_size_t, _P]),
    "gstex_loss_bwd": (c_int32, [c_int32, c_int32, c_int32, _P, _P, _P, _P, _P, POINTER(c_float), c_float, _P, _P,
                                 _P, _P, _P, c_size_t, _P]),
    "gstex_adam_step": (c_int32, [c_int32, POINTER(GstexAdamTensor), c_double, c_double, c_double, _P]),
    "gstex_adam_step_ex": (c_int32, [c_int32, POINTER(GstexAdamTensor), c_double, c_double, c_double, c_int32, _P]),
    "gstex_adam_step_scaled": (c_int32, [c_int32, POINTER(GstexAdamTensor), c_double, c_double, c_double, c_int32,
                                         c_float, _P]),
    "gstex_adam_step_guarded": (c_int32, [c_int32, POINTER(GstexAdamTensor), c_double, c_double, c_double, c_int32,
                                          c_float, _P, _P]),
    "gstex_train_prologue": (c_int32, [POINTER(GstexTrainPrologueArgs), _P]),
    "gstex_train_prologue_scan_bytes": (c_size_t, [c_int32]),
    "gstex_train_epilogue": (c_int32, [POINTER(GstexTrainEpilogueArgs), _P]),
}

_lib = None
_lock = threading.Lock()


class GstexError(RuntimeError):
    pass


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and return the C-ABI library; raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise GstexError(
                    f"{path} is missing: build it with `make -C gstex_amd/csrc` "
                    "(or `python -c 'import __graft_entry__ as g; g.build()'`). "
                    "gstex_amd has no CPU fallback."
                )
            lib = ctypes.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def last_error() -> str:
    msg = load().gstex_last_error()
    return msg.decode() if msg else ""


def call(name: str, *args) -> None:
    """Call a status-returning entry point; raise GstexError with the library's message."""
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise GstexError(f"{name} failed (status {rc}): {last_error()}")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None / empty)."""
    if t is None:
        return None
    if t.numel() == 0:
        return None
    return t.data_ptr()


def stream_of(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class _Event:
    __slots__ = ("_h",)
    KIND = 0

    def __init__(self):
        h = c_void_p()
        call("gstex_event_create", self.KIND, ctypes.byref(h))
        self._h = h.value

    def record(self, device=None, stream: int | None = None) -> None:
        """Record on `stream` (a HIP stream handle), default the current stream of `device`."""
        call("gstex_event_record", self._h, stream if stream is not None else torch.cuda.current_stream(device).cuda_stream)

    @property
    def handle(self) -> int:
        return self._h

    def __del__(self):
        try:
            if self._h:
                load().gstex_event_destroy(self._h)
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass


class TimingEvent(_Event):
    """A HIP event for timing only (gstex_event_create(GSTEX_EVENT_TIMING), ABI 14: no system-scope fence when
    recorded, so a pair around a kernel does not write back and invalidate the caches between launches);
    elapsed_time(end) in ms once both have completed."""

    __slots__ = ()
    KIND = 0

    def elapsed_time(self, end: "TimingEvent") -> float:
        ms = c_float()
        call("gstex_event_elapsed", self._h, end._h, ctypes.byref(ms))
        return float(ms.value)


class OrderEvent(_Event):
    """A HIP event for ordering one stream after another on the same device (GSTEX_EVENT_ORDER: no timing, a
    device-scope release instead of the default event's system-scope one); wait(stream) = hipStreamWaitEvent."""

    __slots__ = ()
    KIND = 1

    def wait(self, device=None, stream: int | None = None) -> None:
        call("gstex_stream_wait_event",
             stream if stream is not None else torch.cuda.current_stream(device).cuda_stream, self._h)


def make_camera(viewmat, c2w, fx, fy, cx, cy, H, W, block) -> GstexCamera:
    """viewmat: device fp32 (3,4) contiguous; c2w: device fp32 (4,4) contiguous or None."""
    return GstexCamera(
        ptr(viewmat), ptr(c2w) if c2w is not None else None,
        float(fx), float(fy), float(cx), float(cy), int(H), int(W), int(block),
    )
