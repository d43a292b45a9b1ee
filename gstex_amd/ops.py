"""torch.autograd front-ends of the libgstex_hip.so C-ABI.

These mirror the `gstex_cuda` Python surface that nerfstudio/models/gstex.py imports
(gstex.py:28-32, models/jagged_texture.py:7-8, scripts/exporter.py:40): same names, positional
arguments and return tuples.  All work is enqueued on torch's current HIP stream.  There is no CPU
path: inputs must be HIP tensors, and a missing library raises (see gstex_amd/_lib.py).
"""
from __future__ import annotations

import ctypes
import os
import time
from typing import NamedTuple, Tuple

import torch

from . import _lib
from ._lib import PARTIAL_FLOATS, PARTIAL_FLOATS_PHOTO, REC_FLOATS, call, ptr

BLOCK_WIDTH = 16
# near-edge-on splats' homogeneous points evaluated from their fp64 setup rows by the raster forward and backward alike
# (gstex_raster_setup / _fwd_zero / _bwd hp_records, ABI 18); GSTEX_HP=0 evaluates every pair from the
# fp32 record (the round-5 numerics)
HP_RECORDS = os.environ.get("GSTEX_HP", "1") != "0"
# diagnostics: called with (partials, row_flags, records, hp rows) after each raster backward (tools/hp_partials.py)
PARTIALS_HOOK = None

# ----------------------------------------------------------------------------------------
# optional per-kernel timing: HIP events recorded on the stream each kernel is launched on
# ----------------------------------------------------------------------------------------
_TIMING: dict | None = None


_TIMED_DEFAULT = ("gstex_raster_fwd", "gstex_raster_bwd")  # the roofline kernels
_TIMED = set(_TIMED_DEFAULT)


def set_kernel_timing(enabled: bool, names=None) -> None:
    """Record a HIP event pair around the raster forward / backward launches (or the C-ABI entry points in
    `names`) on the stream they run on (bench.py / profiling only)."""
    global _TIMING, _TIMED
    _TIMING = {} if enabled else None
    _TIMED = set(names) if names is not None else set(_TIMED_DEFAULT)


def kernel_times() -> dict:
    """{name: [ms, ...]} for the launches recorded since set_kernel_timing(True) (synchronises)."""
    if not _TIMING:
        return {}
    torch.cuda.synchronize()
    return {k: [a.elapsed_time(b) for a, b in v] for k, v in _TIMING.items()}


def _TIMING_EVENTS(name: str) -> list:
    """The (start, end) HIP event pairs recorded for `name` since set_kernel_timing(True) (no synchronisation)."""
    return list((_TIMING or {}).get(name, []))


def _launch(name: str, *args) -> None:
    # gstex_raster_fwd_zero times as the forward
    key = name[:-len("_zero")] if name.endswith("_zero") else name
    if _TIMING is None or key not in _TIMED or torch.cuda.is_current_stream_capturing():
        call(name, *args)
        return
    # fence-free timing events (_lib.TimingEvent): a default event pair around each launch cost ~10 us of device time
    a = _lib.TimingEvent()
    b = _lib.TimingEvent()
    a.record()
    call(name, *args)
    b.record()
    _TIMING.setdefault(key, []).append((a, b))


# ----------------------------------------------------------------------------------------
# validation helpers (TORCH_CHECK-style RuntimeErrors)
# ----------------------------------------------------------------------------------------
def _check(cond: bool, msg: str) -> None:
    if not cond:
        raise RuntimeError(msg)


def _dev(t: torch.Tensor, name: str) -> None:
    _check(isinstance(t, torch.Tensor), f"{name} must be a tensor")
    _check(t.is_cuda, f"{name} must be a HIP (cuda) tensor; gstex_amd has no CPU path (got {t.device})")


def _f32(t: torch.Tensor, name: str, shape=None) -> torch.Tensor:
    _dev(t, name)
    _check(t.dtype == torch.float32, f"{name} must be float32 (got {t.dtype})")
    if shape is not None:
        _check(t.dim() == len(shape) and all(s is None or s == d for s, d in zip(shape, t.shape)),
               f"{name} must have shape {tuple('*' if s is None else s for s in shape)} (got {tuple(t.shape)})")
    return t.contiguous()


def _i32(t: torch.Tensor, name: str, shape=None) -> torch.Tensor:
    _dev(t, name)
    _check(t.dtype == torch.int32, f"{name} must be int32 (got {t.dtype})")
    if shape is not None:
        _check(t.dim() == len(shape) and all(s is None or s == d for s, d in zip(shape, t.shape)),
               f"{name} must have shape {tuple('*' if s is None else s for s in shape)} (got {tuple(t.shape)})")
    return t.contiguous()


def _viewmat(viewmat: torch.Tensor) -> torch.Tensor:
    v = viewmat.detach()
    if v.dim() == 3:
        v = v.squeeze(0)
    _check(v.shape in ((3, 4), (4, 4)), f"viewmat must be (3,4) or (4,4) (got {tuple(viewmat.shape)})")
    return _f32(v[:3, :], "viewmat")


def _c2w(c2w) -> torch.Tensor | None:
    if c2w is None:
        return None
    c = c2w.detach()
    if c.dim() == 3:
        c = c.squeeze(0)
    _check(c.shape == (4, 4), f"c2w must be (4,4) (got {tuple(c2w.shape)})")
    return _f32(c, "c2w")


def _stream(t: torch.Tensor) -> int:
    return _lib.stream_of(t.device)


# ----------------------------------------------------------------------------------------
# project_points / get_aabb_2d / get_num_tiles_hit_2d
# ----------------------------------------------------------------------------------------
class _ProjectPoints(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means, viewmat, fx, fy, cx, cy):
        means = _f32(means, "means", (None, 3))
        vm = _viewmat(viewmat)
        n = means.shape[0]
        xys = torch.empty((n, 2), device=means.device, dtype=torch.float32)
        depths = torch.empty((n,), device=means.device, dtype=torch.float32)
        cam = _lib.make_camera(vm, None, fx, fy, cx, cy, 0, 0, BLOCK_WIDTH)
        call("gstex_project_points", n, ptr(means), cam, ptr(xys), ptr(depths), _stream(means))
        ctx.save_for_backward(means, vm)
        ctx.intr = (fx, fy, cx, cy)
        ctx.set_materialize_grads(False)  # the kernel reads a NULL v_xys / v_depths as zero
        return xys, depths

    @staticmethod
    def backward(ctx, v_xys, v_depths):
        if v_xys is None and v_depths is None:
            # reached with no upstream gradient (texture_gaussians uses depths only as sort keys): the
            # gradient is exactly zero, so none is returned (no kernel, no accumulation into means.grad)
            return None, None, None, None, None, None
        means, vm = ctx.saved_tensors
        n = means.shape[0]
        v_means = torch.empty_like(means)
        cam = _lib.make_camera(vm, None, *ctx.intr, 0, 0, BLOCK_WIDTH)
        v_xys = v_xys.contiguous() if v_xys is not None else None
        v_depths = v_depths.contiguous() if v_depths is not None else None
        call("gstex_project_points_bwd", n, ptr(means), cam, ptr(v_xys), ptr(v_depths), ptr(v_means),
             _stream(means))
        return v_means, None, None, None, None, None


def project_points(means: torch.Tensor, viewmat: torch.Tensor, intrinsics) -> Tuple[torch.Tensor, torch.Tensor]:
    """Pinhole projection of splat centres -> (xys (N,2), depths (N,)). gstex.py:1077."""
    fx, fy, cx, cy = [float(v) for v in intrinsics]
    return _ProjectPoints.apply(means, viewmat, fx, fy, cx, cy)


class _Aabb2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means, scales, glob_scale, quats, viewmat, fx, fy, cx, cy):
        means = _f32(means, "means", (None, 3))
        n = means.shape[0]
        scales = _f32(scales, "scales", (n, 3))
        quats = _f32(quats, "quats", (n, 4))
        vm = _viewmat(viewmat)
        centers = torch.empty((n, 2), device=means.device, dtype=torch.float32)
        extents = torch.empty((n, 2), device=means.device, dtype=torch.float32)
        cam = _lib.make_camera(vm, None, fx, fy, cx, cy, 0, 0, BLOCK_WIDTH)
        call("gstex_aabb_2d", n, ptr(means), ptr(scales), float(glob_scale), ptr(quats), cam, ptr(centers),
             ptr(extents), _stream(means))
        ctx.save_for_backward(means, scales, quats, vm)
        ctx.args = (float(glob_scale), fx, fy, cx, cy)
        ctx.mark_non_differentiable(extents)
        ctx.set_materialize_grads(False)
        return centers, extents

    @staticmethod
    def backward(ctx, v_centers, v_extents):
        means, scales, quats, vm = ctx.saved_tensors
        glob, fx, fy, cx, cy = ctx.args
        n = means.shape[0]
        if v_centers is None:
            return None, None, None, None, None, None, None, None, None
        v_means = torch.empty_like(means)  # written in full by the kernel
        v_scales = torch.empty_like(scales)
        v_quats = torch.empty_like(quats)
        cam = _lib.make_camera(vm, None, fx, fy, cx, cy, 0, 0, BLOCK_WIDTH)
        call("gstex_aabb_2d_bwd", n, ptr(means), ptr(scales), glob, ptr(quats), cam,
             ptr(v_centers.contiguous()), ptr(v_means), ptr(v_scales), ptr(v_quats), _stream(means))
        return v_means, v_scales, None, v_quats, None, None, None, None, None


def get_aabb_2d(means, scales, glob_scale, quats, viewmat, intrinsics):
    """2DGS screen-space bound -> (centers (N,2), extents (N,2)). gstex.py:1079."""
    fx, fy, cx, cy = [float(v) for v in intrinsics]
    return _Aabb2d.apply(means, scales, glob_scale, quats, viewmat, fx, fy, cx, cy)


def get_num_tiles_hit_2d(centers, extents, H: int, W: int, block_width: int) -> torch.Tensor:
    """Tiles overlapped by centre +- extent (gsplat-0.1 tile-bbox convention) -> int32 (N,).
    gstex.py:1080."""
    centers = _f32(centers.detach(), "centers", (None, 2))
    n = centers.shape[0]
    extents = _f32(extents.detach(), "extents", (n, 2))
    out = torch.empty((n,), device=centers.device, dtype=torch.int32)
    call("gstex_num_tiles_hit", n, ptr(centers), ptr(extents), int(H), int(W), int(block_width), ptr(out),
         _stream(centers))
    return out


def preprocess(means, scales, glob_scale, quats, viewmat, intrinsics, H: int, W: int):
    """project_points' depths, get_aabb_2d and get_num_tiles_hit_2d in one launch (gstex_preprocess) ->
    (depths (N,), centers (N,2), extents (N,2), num_tiles_hit (N,) int32), bit-identical to the three calls and
    without autograd: for texture_gaussians(..., fold_aabb=True), whose backward chains the centre gradient itself
    (the training path; gstex.py:1077-1080)."""
    fx, fy, cx, cy = [float(v) for v in intrinsics]
    means = _f32(means.detach(), "means", (None, 3))
    n = means.shape[0]
    scales = _f32(scales.detach(), "scales", (n, 3))
    quats = _f32(quats.detach(), "quats", (n, 4))
    vm = _viewmat(viewmat)
    f = dict(device=means.device, dtype=torch.float32)
    depths = torch.empty((n,), **f)
    centers = torch.empty((n, 2), **f)
    extents = torch.empty((n, 2), **f)
    nth = torch.empty((n,), device=means.device, dtype=torch.int32)
    cam = _lib.make_camera(vm, None, fx, fy, cx, cy, H, W, BLOCK_WIDTH)
    call("gstex_preprocess", n, ptr(means), ptr(scales), float(glob_scale), ptr(quats), cam, ptr(depths),
         ptr(centers), ptr(extents), ptr(nth), _stream(means))
    return depths, centers, extents, nth


# ----------------------------------------------------------------------------------------
# binning
# ----------------------------------------------------------------------------------------
_PINNED = {}
_ZEROS = {}


def _zero_scalar(device) -> torch.Tensor:
    """One cached fp32 zero per device, the storage of the geometry outputs a photometric forward does not
    produce (returned as broadcast views)."""
    key = str(device)
    z = _ZEROS.get(key)
    if z is None:
        z = _ZEROS[key] = torch.zeros((), device=device, dtype=torch.float32)
    return z


def _start_count(x: torch.Tensor):
    """Queue the copy of a non-negative int32 device scalar into a pinned host word preset to -1 (stream-ordered);
    _finish_count polls that word.  Work queued between the two calls runs on the device while the host waits
    and then sizes buffers from the value, instead of the device idling through that host time."""
    buf = _PINNED.get(x.device)
    if buf is None:
        buf = _PINNED[x.device] = torch.empty((1,), dtype=torch.int32, pin_memory=True)
    host = buf.numpy()
    host[0] = -1
    buf.copy_(x.reshape(1), non_blocking=True)
    return host, x.device


def _finish_count(pending) -> int:
    """Host value of a _start_count copy: polls the pinned word, which returns as soon as the copy lands instead
    of after a blocking stream synchronisation's wake-up (~50 us of idle GPU per step, measured).  After 50 ms
    without the copy it falls back to a real synchronisation (which raises any pending device error)."""
    host, dev = pending
    deadline = None
    while host[0] < 0:
        if deadline is None:
            deadline = time.perf_counter() + 0.05
        elif time.perf_counter() > deadline:
            torch.cuda.current_stream(dev).synchronize()
            break
    return int(host[0])


def _read_count(x: torch.Tensor) -> int:
    return _finish_count(_start_count(x))


def bin_begin(num_tiles_hit):
    """First half of bin_and_sort: the offsets scan and the asynchronous read of the pair count."""
    n = num_tiles_hit.shape[0]
    dev = num_tiles_hit.device
    nth = _i32(num_tiles_hit, "num_tiles_hit", (n,))
    offsets = torch.empty((n + 1,), device=dev, dtype=torch.int32)
    ws = torch.empty((max(int(_lib.load().gstex_scan_workspace_size(n)), 1),), device=dev, dtype=torch.uint8)
    call("gstex_scan_offsets", n, ptr(nth), ptr(offsets), ptr(ws), ws.numel(), _stream(nth))
    pending = _start_count(offsets[n]) if offsets.is_cuda else int(offsets[n].item())
    return nth, offsets, pending


def bin_finish(begun, centers, extents, depths, H: int, W: int, block_width: int = BLOCK_WIDTH,
               with_order: bool = False):
    """Second half of bin_and_sort: wait for the pair count, size the pair buffers, bin and sort.  with_order:
    also return the largest-first tile order the sort ranked (gstex_bin_sort_ordered; == tile_order(ranges))."""
    nth, offsets, pending = begun
    n = nth.shape[0]
    dev = nth.device
    st = _stream(nth)
    n_isect = pending if isinstance(pending, int) else _finish_count(pending)
    tiles_x = (W + block_width - 1) // block_width
    tiles_y = (H + block_width - 1) // block_width
    n_tiles = tiles_x * tiles_y
    tile_ranges = torch.empty((n_tiles, 2), device=dev, dtype=torch.int32)
    sorted_ids = torch.empty((n_isect,), device=dev, dtype=torch.int32)
    sorted_slots = torch.empty((n_isect,), device=dev, dtype=torch.int32)
    wsb = int(_lib.load().gstex_bin_workspace_size(n, n_isect, n_tiles))
    bws = torch.empty((max(wsb, 1),), device=dev, dtype=torch.uint8)
    keep = [t.detach().contiguous() for t in (centers, extents, depths)]  # alive until the launch returns
    geo = (ptr(keep[0]), ptr(keep[1]), ptr(keep[2]), ptr(nth), ptr(offsets), int(H), int(W), int(block_width),
           ptr(tile_ranges), ptr(sorted_ids), ptr(sorted_slots))
    if not with_order:
        _launch("gstex_bin_sort", n, n_isect, *geo, ptr(bws), bws.numel(), st)
        return offsets, tile_ranges, sorted_ids, sorted_slots
    order = torch.empty((n_tiles,), device=dev, dtype=torch.int32)
    _launch("gstex_bin_sort_ordered", n, n_isect, *geo, ptr(order), ptr(bws), bws.numel(), st)
    return offsets, tile_ranges, sorted_ids, sorted_slots, order


class PairCapacity:
    """Read-back-free pair buffers for a training loop (ABI 13; replaces the per-render pair-count read-back of
    gstex.py:1045-1052, 1127 -- a device-to-host copy and a wait on it -- with buffers sized from a capacity).

    Every render's scan writes its pair total on the device (gstex_scan_offsets_guarded): into the step's guard flag
    (1.0 when the total exceeds the capacity; the binning then leaves every tile empty and the guarded Adam skips the
    step's update, gstex_adam_step_guarded) and into one of RING device-writable host words, followed by a
    system-scope fence.  The host sets a slot's word to SENTINEL before the render is enqueued and reads the total once
    the word has changed -- no event in the stream (a recorded event cost ~5 us of device time per render), no copy, no
    synchronisation.  The capacity starts from one read-back of the first render's total (headroom x total + slack)
    and grows when a total comes back above grow_at of it, so an overflow needs a jump of more than 1 / grow_at in the
    total within the few renders the host runs ahead; one that happens anyway skips that step's update (parameters
    and moments untouched, the step counters still advance, identically on every rank) and is recorded in
    `overflows`."""

    RING = 8
    SENTINEL = -(1 << 31)  # (a pair total is >= 0)
    WAIT_S = 10.0  # a slot still unwritten after this long: the stream is synchronised once, then the word must be set

    def __init__(self, device, capacity: int = 0, headroom: float = 1.5, slack: int = 1 << 16, grow_at: float = 0.8):
        self.device = torch.device(device)
        self.capacity = int(capacity)
        self.headroom, self.slack, self.grow_at = float(headroom), int(slack), float(grow_at)
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        call("gstex_host_words_alloc", self.RING, ctypes.byref(h), ctypes.byref(d))
        self._host_ptr, self._dev_ptr = h.value, d.value
        self._words = (ctypes.c_int32 * self.RING).from_address(self._host_ptr)
        self._pending = [False] * self.RING
        self._caps = [0] * self.RING
        self._tags = [None] * self.RING
        self._k = 0
        self.max_total = 0
        self.last_total = None
        self.overflows = []  # tags (trainer steps) of renders whose total exceeded the capacity

    def __del__(self):
        try:
            if self._host_ptr:
                if any(self._pending):  # a scan may still write its word
                    torch.cuda.synchronize(self.device)
                _lib.load().gstex_host_words_free(self._host_ptr)
                self._host_ptr = None
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass

    def _absorb(self, k):
        total = int(self._words[k])
        self._pending[k] = False
        self.last_total = total
        self.max_total = max(self.max_total, total)
        if total > self._caps[k]:
            self.overflows.append(self._tags[k])
        if total > self.grow_at * self.capacity:
            self.capacity = max(self.capacity, int(self.headroom * total) + self.slack)

    def _wait(self, k):
        """Spin until slot k's scan has written its word (the host is RING renders ahead, or the first render)."""
        t0 = time.perf_counter()
        while self._words[k] == self.SENTINEL:
            if time.perf_counter() - t0 > self.WAIT_S:
                torch.cuda.synchronize(self.device)
                if self._words[k] == self.SENTINEL:
                    raise RuntimeError("PairCapacity: a finished scan did not report its pair total")
                break
        self._absorb(k)

    def poll(self):
        """Read the totals of the renders the device has scanned (non-blocking); returns the number of overflows."""
        before = len(self.overflows)
        for k in range(self.RING):
            if self._pending[k] and self._words[k] != self.SENTINEL:
                self._absorb(k)
        return len(self.overflows) - before

    def scan(self, nth: torch.Tensor, step_flag: torch.Tensor, first: bool, tag=None):
        """The offsets scan of one render with the guard: -> (offsets (n+1,), capacity for this render)."""
        n = nth.shape[0]
        guard, k, cap = self.reserve(step_flag, first, tag, sized=False)
        offsets = torch.empty((n + 1,), device=nth.device, dtype=torch.int32)
        ws = torch.empty((max(int(_lib.load().gstex_scan_workspace_size(n)), 1),), device=nth.device, dtype=torch.uint8)
        call("gstex_scan_offsets_guarded", n, ptr(nth), ptr(offsets), ptr(ws), ws.numel(), ctypes.byref(guard),
             _stream(nth))
        return offsets, self.commit(k, cap, tag, nth.device)

    def reserve(self, step_flag: torch.Tensor, first: bool, tag=None, sized: bool = True):
        """The guard of one render's scan and its ring slot -> (GstexPairGuard, slot, capacity of the render).  The
        caller launches the guarded scan, then commit()s the slot.  sized=True (gstex_amd.fused, which sizes its
        buffers before the scan) requires the capacity to have been set by an earlier render."""
        if sized and self.capacity <= 0:
            raise RuntimeError("PairCapacity.reserve: no capacity yet (the first render sizes it through scan())")
        k = self._k % self.RING
        if self._pending[k]:  # the host is RING renders ahead: wait for that one (normally long done)
            self._wait(k)
        self._k += 1
        cap = (1 << 62) if self.capacity <= 0 else self.capacity
        self._words[k] = self.SENTINEL  # (stored before the scan is enqueued; the scan overwrites it)
        self._pending[k], self._caps[k], self._tags[k] = True, cap, tag
        return _lib.GstexPairGuard(cap, ptr(step_flag), self._dev_ptr + 4 * k, 1 if first else 0), k, cap

    def commit(self, k: int, cap: int, tag, device) -> int:
        """After slot k's scan has been enqueued: the first render reads its total back and sizes the capacity.
        -> the capacity."""
        if self.capacity <= 0:  # the one read-back: the first render sizes the capacity
            self._wait(k)
            self.capacity = max(self.capacity, int(self.headroom * self.last_total) + self.slack)
        return self.capacity


def bin_capped(nth, offsets, capacity: int, centers, extents, depths, H: int, W: int, block_width: int = BLOCK_WIDTH):
    """bin_finish without the host's pair count: buffers of `capacity` pairs, the total read on the device
    (gstex_bin_sort_capped).  -> (offsets, tile_ranges, sorted_ids (capacity,), sorted_slots (capacity,), order)."""
    n = nth.shape[0]
    dev = nth.device
    tiles_x = (W + block_width - 1) // block_width
    tiles_y = (H + block_width - 1) // block_width
    n_tiles = tiles_x * tiles_y
    tile_ranges = torch.empty((n_tiles, 2), device=dev, dtype=torch.int32)
    sorted_ids = torch.empty((capacity,), device=dev, dtype=torch.int32)
    sorted_slots = torch.empty((capacity,), device=dev, dtype=torch.int32)
    order = torch.empty((n_tiles,), device=dev, dtype=torch.int32)
    bws = torch.empty((max(int(_lib.load().gstex_bin_workspace_size(n, capacity, n_tiles)), 1),), device=dev,
                      dtype=torch.uint8)
    keep = [t.detach().contiguous() for t in (centers, extents, depths)]
    _launch("gstex_bin_sort_capped", n, capacity, ptr(keep[0]), ptr(keep[1]), ptr(keep[2]), ptr(nth), ptr(offsets),
            int(H), int(W), int(block_width), ptr(tile_ranges), ptr(sorted_ids), ptr(sorted_slots), ptr(order),
            ptr(bws), bws.numel(), _stream(nth))
    return offsets, tile_ranges, sorted_ids, sorted_slots, order


def bin_and_sort(centers, extents, depths, num_tiles_hit, H: int, W: int, block_width: int = BLOCK_WIDTH):
    """Tile binning + per-tile depth sort.  Returns (offsets (N+1,), tile_ranges (n_tiles,2),
    sorted_ids (I,), sorted_slots (I,)), all int32.  One host read of the pair count I to size the I-length
    buffers."""
    _i32(num_tiles_hit, "num_tiles_hit", (centers.shape[0],))
    return bin_finish(bin_begin(num_tiles_hit), centers, extents, depths, H, W, block_width)


def tile_order(tile_ranges: torch.Tensor) -> torch.Tensor:
    """Largest-first raster launch order (int32 (n_tiles,)) from bin_and_sort's tile_ranges."""
    tr = _i32(tile_ranges, "tile_ranges", (None, 2))
    order = torch.empty((tr.shape[0],), device=tr.device, dtype=torch.int32)
    call("gstex_tile_order", tr.shape[0], ptr(tr), ptr(order), _stream(tr))
    return order


def unit_order(unit_cost: torch.Tensor) -> torch.Tensor:
    """gstex_unit_order: the backward's launch order from unit keys (cost | XCD group << 24), computed inside
    gstex_raster_bwd; exposed for tests.  -1 at positions no unit takes."""
    uc = _i32(unit_cost, "unit_cost", (None,))
    order = torch.empty_like(uc)
    scratch = torch.empty((int(_lib.load().gstex_unit_order_scratch_words()),), device=uc.device, dtype=torch.int32)
    call("gstex_unit_order", uc.shape[0], ptr(uc), ptr(order), ptr(scratch), _stream(uc))
    return order


# ----------------------------------------------------------------------------------------
# texture_gaussians
# ----------------------------------------------------------------------------------------
class _TextureGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, texture_info, texture_dims, centers, extents, depths, num_tiles_hit, rgbs, opacities, means,
                scales, glob_scale, quats, uv0, umap, vmap, texture, viewmat, c2w, fx, fy, cx, cy, H, W,
                block_width, settings, background, texture_transform=None, fold_aabb=False,
                geometry_outputs=True, grad_enabled=True, texture_grad_sink=None, on_texture_grad=None,
                texture_ready=None, binning=None, before_pair_wait=None, zero_sink=False, pair_guard=None):
        N, L, C = (int(v) for v in texture_info)
        _check(L == 1, f"texture_info[1] (texture layers) must be 1 (got {L})")
        _check(1 <= C <= 8, f"texture_info[2] (channels) must be in [1, 8] (got {C})")
        _check(int(block_width) == BLOCK_WIDTH, f"block_width must be {BLOCK_WIDTH} (got {block_width})")
        means = _f32(means, "means", (None, 3))
        n = means.shape[0]
        _check(N == n, f"texture_info[0] ({N}) != number of splats ({n})")
        dims = _i32(texture_dims, "texture_dims", (n, 3))
        centers_c = _f32(centers, "centers", (n, 2))
        extents_c = _f32(extents.detach(), "extents", (n, 2))
        depths_c = _f32(depths.detach(), "depths", (n,))
        nth = _i32(num_tiles_hit, "num_tiles_hit", (n,))
        rgbs = _f32(rgbs, "rgbs", (n, 3))
        opacities = _f32(opacities, "opacities", (n, 1))
        scales = _f32(scales, "scales", (n, 3))
        quats = _f32(quats, "quats", (n, 4))
        uv0 = _f32(uv0, "uv0", (n, 1, 2))
        umap = _f32(umap, "umap", (n, 1, 3))
        vmap = _f32(vmap, "vmap", (n, 1, 3))
        texture = _f32(texture, "texture", (None, C))
        vm = _viewmat(viewmat)
        cw = _c2w(c2w)
        bg = _f32(background.detach(), "background", (3,)) if background is not None else None
        H, W = int(H), int(W)
        dev = means.device
        st = _stream(means)
        cam = _lib.make_camera(vm, cw, fx, fy, cx, cy, H, W, BLOCK_WIDTH)

        # the pair count is read to the host once; work that does not depend on the tile lists is queued
        # between the copy and the wait, so the device runs it while the host waits and sizes the pair
        # buffers: the splat records and the zeroed texel-gradient buffer of the backward
        capped = None
        if binning is None and pair_guard is not None:  # capacity mode: no host read of the pair total
            pcap, step_flag, first, tag = pair_guard
            capped = pcap.scan(nth, step_flag, first, tag)
        begun = bin_begin(nth) if binning is None and capped is None else None
        records = torch.empty((n, REC_FLOATS), device=dev, dtype=torch.float32)
        # backward-only buffers only when a backward can follow: not under torch.no_grad() (eval renders of
        # trainable parameters), where apply() records no graph whatever the inputs' requires_grad
        needs_bwd = bool(grad_enabled) and any(ctx.needs_input_grad)
        # the near-edge-on splats' fp64 rows (read by the forward and the backward)
        hp = torch.empty((n, _lib.HP_DOUBLES), device=dev, dtype=torch.float64) if HP_RECORDS else None
        _launch("gstex_raster_setup", n, ptr(means), ptr(scales), float(glob_scale), ptr(quats), ptr(rgbs),
                ptr(opacities), ptr(centers_c), ptr(uv0), ptr(umap), ptr(vmap), ptr(dims), ptr(nth), cam,
                ptr(records), ptr(hp), st)
        ctx.hp = hp
        ctx.v_texture = None
        ctx.sink = texture_grad_sink is not None
        ctx.on_texture_grad = on_texture_grad
        if needs_bwd and ctx.needs_input_grad[15]:
            if ctx.sink:  # the caller's gradient buffer: zeroed by the raster forward, accumulated into by the
                # backward, nothing returned to autograd
                _check(texture_grad_sink.shape == texture.shape and texture_grad_sink.is_contiguous() and
                       texture_grad_sink.dtype == torch.float32 and texture_grad_sink.device == texture.device,
                       "texture_grad_sink must be a contiguous fp32 tensor shaped like texture on its device")
                ctx.v_texture = texture_grad_sink
            else:
                ctx.v_texture = torch.empty_like(texture)  # zeroed by the raster forward (gstex_raster_fwd_zero)
        if before_pair_wait is not None:
            before_pair_wait()  # caller's work for the device while the host waits for the pair count
        if capped is not None:
            offsets, tile_ranges, sorted_ids, sorted_slots, order = bin_capped(
                nth, capped[0], capped[1], centers_c.detach(), extents_c, depths_c, H, W, BLOCK_WIDTH)
        elif binning is None:
            offsets, tile_ranges, sorted_ids, sorted_slots, order = bin_finish(
                begun, centers_c.detach(), extents_c, depths_c, H, W, BLOCK_WIDTH, with_order=True)
        else:  # a previous call's binning of the same centres / extents / depths / num_tiles_hit (bin_gaussians)
            _check(binning.n == n and binning.H == H and binning.W == W and binning.nth.data_ptr() == nth.data_ptr(),
                   "binning was computed for other splats / image size / num_tiles_hit")
            offsets, tile_ranges, sorted_ids, sorted_slots, order = (binning.offsets, binning.tile_ranges,
                                                                     binning.sorted_ids, binning.sorted_slots,
                                                                     binning.order)
        ctx_scale, ctx_bias = (1.0, 0.0) if texture_transform is None else (float(texture_transform[0]),
                                                                             float(texture_transform[1]))
        f = dict(device=dev, dtype=torch.float32)
        img = torch.empty((H, W, 3), **f)
        alpha = torch.empty((H, W), **f)
        tex = torch.empty((H, W, C), **f)
        state = torch.empty((H, W, 4), **f)
        if geometry_outputs:
            depth = torch.empty((H, W), **f)
            reg = torch.empty((H, W), **f)
            normal = torch.empty((H, W, 3), **f)
            geo_ptrs = (ptr(depth), ptr(reg), ptr(normal))
            if int(settings) & _lib.SETTING_EVAL_NORMAL:
                ctx.mark_non_differentiable(normal)  # bit 15: unit normals, a forward-only eval output
        else:  # not produced by the kernel: zeros, no gradient (read-only broadcast views of one cached zero:
            # no fill per call; an in-place write into them raises instead of corrupting later calls)
            z = _zero_scalar(f["device"])
            depth, reg, normal = z.expand(H, W), z.expand(H, W), z.expand(H, W, 3)
            geo_ptrs = (None, None, None)
            ctx.mark_non_differentiable(depth, reg, normal)
        # per (tile, wave, splat) cull bits of the forward for the backward
        # the forward's record for the backward (cull bits, per-unit costs, checkpoints of deep tile lists)
        aux = None
        n_isect = sorted_ids.shape[0]
        if needs_bwd:
            nb = int(_lib.load().gstex_raster_aux_bytes(n_isect, tile_ranges.shape[0], C))
            aux = torch.empty((nb,), device=dev, dtype=torch.uint8)
        if callable(texture_ready):  # the caller's texel update, enqueued right before the raster forward
            texture_ready()
        elif texture_ready is not None:  # the texels (and the gradient buffer) are updated on another stream
            torch.cuda.current_stream(dev).wait_event(texture_ready)
        # the buffers the backward accumulates into are zeroed by the forward's grid (no fill passes): the texel
        # gradient (this call's own buffer, or the caller's sink when zero_sink) and the fast mode's per-splat partial
        # sums (PARTIAL_FLOATS per splat: room for either row width)
        zbuf = ctx.v_texture if (not ctx.sink or zero_sink) else None
        ctx.partials = torch.empty((n * PARTIAL_FLOATS,), device=dev, dtype=torch.float32) if needs_bwd else None
        _launch("gstex_raster_fwd_zero", cam, C, int(settings), ptr(bg), ptr(records), ptr(hp), ptr(tile_ranges),
                ptr(order),
             ptr(sorted_ids),
             ptr(texture), texture.shape[0], ctx_scale, ctx_bias, ptr(img), geo_ptrs[0], geo_ptrs[1], ptr(alpha),
             ptr(tex), geo_ptrs[2],
             ptr(state), n_isect, ptr(aux), ptr(zbuf), 0 if zbuf is None else zbuf.numel(), ptr(ctx.partials),
             0 if ctx.partials is None else ctx.partials.numel(), st)
        ctx.aux = aux
        ctx.save_for_backward(means, scales, quats, opacities, umap, vmap, texture, nth, offsets, tile_ranges,
                              order, sorted_ids, sorted_slots, records, state, vm, cw if cw is not None else vm,
                              bg if bg is not None else vm)
        ctx.has_c2w = cw is not None
        ctx.has_bg = bg is not None
        ctx.args = (float(glob_scale), float(fx), float(fy), float(cx), float(cy), H, W, C, int(settings))
        ctx.tex_affine = (ctx_scale, ctx_bias)
        ctx.fold_aabb = bool(fold_aabb)
        ctx.set_materialize_grads(False)  # unused outputs' gradients stay None (no zero tensors)
        return img, depth, reg, alpha, tex, normal

    @staticmethod
    def backward(ctx, v_img, v_depth, v_reg, v_alpha, v_tex, v_normal):
        (means, scales, quats, opacities, umap, vmap, texture, nth, offsets, tile_ranges, order, sorted_ids,
         sorted_slots, records, state, vm, cw, bg) = ctx.saved_tensors
        cw = cw if ctx.has_c2w else None
        bg = bg if ctx.has_bg else None
        glob, fx, fy, cx, cy, H, W, C, settings = ctx.args
        n = means.shape[0]
        dev = means.device
        st = _stream(means)
        cam = _lib.make_camera(vm, cw, fx, fy, cx, cy, H, W, BLOCK_WIDTH)

        def g(t, shape):  # unused outputs arrive as None (no zero fill): the kernel reads NULL as zero
            return None if t is None else t.contiguous()

        v_img = g(v_img, (H, W, 3))
        v_depth = g(v_depth, (H, W))
        v_reg = g(v_reg, (H, W))
        v_alpha = g(v_alpha, (H, W))
        v_tex = g(v_tex, (H, W, C))
        v_normal = g(v_normal, (H, W, 3))
        n_isect = sorted_ids.shape[0]
        # 24 values per (pair, quadrant) sum without depth / normal / distortion gradients (gstex_raster_bwd), 32 with.
        # Default: float-atomic accumulation per splat (like the texel gradients).  Under
        # torch.use_deterministic_algorithms(True): one row per (pair, 8x8 quadrant), written only where the quadrant
        # contributes (row_flags), summed in a fixed order by setup_bwd -- bitwise reproducible splat gradients
        geo = v_depth is not None or v_normal is not None or (v_reg is not None and bool(settings & (1 << 10)))
        row_floats = PARTIAL_FLOATS if geo else PARTIAL_FLOATS_PHOTO
        if torch.are_deterministic_algorithms_enabled():
            partials = torch.empty((n_isect, 4, row_floats), device=dev, dtype=torch.float32)
            row_flags = torch.empty((n_isect,), device=dev, dtype=torch.int32)
        elif ctx.partials is not None:  # zeroed by the forward (a second backward of the same graph zeroes its own)
            partials = ctx.partials[:n * row_floats].view(n, row_floats)
            ctx.partials = None
            row_flags = None
        else:
            partials = torch.zeros((n, row_floats), device=dev, dtype=torch.float32)
            row_flags = None
        v_texture = ctx.v_texture if ctx.v_texture is not None else torch.zeros_like(texture)
        ctx.v_texture = None
        _launch("gstex_raster_bwd", cam, C, int(settings), ptr(bg), ptr(records), ptr(ctx.hp),
                ptr(tile_ranges),
                ptr(sorted_ids), ptr(sorted_slots), ptr(texture), texture.shape[0], ctx.tex_affine[0],
                ctx.tex_affine[1], ptr(state), ptr(v_img), ptr(v_depth), ptr(v_reg), ptr(v_alpha), ptr(v_tex),
                ptr(v_normal), n_isect, ptr(partials), ptr(row_flags), ptr(v_texture), ptr(ctx.aux), st)
        if PARTIALS_HOOK is not None:  # diagnostics (tools/hp_partials.py): the per-splat sums before the chain
            PARTIALS_HOOK(partials, row_flags, records, ctx.hp)
        ctx.aux = None
        ctx.hp = None
        if ctx.sink:
            if ctx.on_texture_grad is not None:
                ctx.on_texture_grad()  # the texel gradient is complete in stream order
            v_texture = None
        v_means = torch.empty_like(means)
        v_scales = torch.empty_like(scales)
        v_quats = torch.empty_like(quats)
        v_rgbs = torch.empty((n, 3), device=dev, dtype=torch.float32)
        v_opac = torch.empty((n, 1), device=dev, dtype=torch.float32)
        v_centers = torch.empty((n, 2), device=dev, dtype=torch.float32)
        v_uv0 = torch.empty((n, 1, 2), device=dev, dtype=torch.float32)
        _launch("gstex_raster_setup_bwd_aabb" if ctx.fold_aabb else "gstex_raster_setup_bwd", n, ptr(means),
                ptr(scales), glob, ptr(quats), ptr(opacities), ptr(umap), ptr(vmap), ptr(nth), ptr(offsets), ptr(partials),
                ptr(row_flags), row_floats, n_isect if row_flags is not None else -1, cam,
                ptr(v_means), ptr(v_scales), ptr(v_quats), ptr(v_rgbs), ptr(v_opac), ptr(v_centers), ptr(v_uv0), st)
        v_bg = None
        if ctx.needs_input_grad[26]:
            v_bg = (v_img * state[..., 0:1]).sum((0, 1)) if v_img is not None else torch.zeros_like(bg)
        if ctx.fold_aabb:
            v_centers = None  # already chained through the AABB centre into v_means / v_scales / v_quats
        return (None, None, v_centers, None, None, None, v_rgbs, v_opac, v_means, v_scales, None, v_quats, v_uv0,
                None, None, v_texture, None, None, None, None, None, None, None, None, None, None, v_bg, None, None,
                None, None, None, None, None, None, None, None, None)


def texture_gaussians(texture_info, texture_dims, centers, extents, depths, num_tiles_hit, rgbs, opacities, means,
                      scales, glob_scale, quats, uv0, umap, vmap, texture, viewmat, c2w, fx, fy, cx, cy, H, W,
                      block_width, settings, background=None, use_torch_impl=False, texture_transform=None,
                      fold_aabb=False, geometry_outputs=True, texture_grad_sink=None, on_texture_grad=None,
                      texture_ready=None, binning=None, before_pair_wait=None, zero_texture_grad_sink=False,
                      pair_guard=None):
    """Differentiable textured-2DGS rasterizer (gstex.py:1133-1162).

    texture_transform=(s, b) (not in the reference API; default None = as stored) makes the raster read
    texel values s * texture + b, so SH2RGB(texture_dc) (gstex.py:1119) need not be materialised: pass
    texture_dc with (0.28209479177387814, 0.5); the texture gradient is then w.r.t. the stored values.

    fold_aabb=True (not in the reference API; training path only) declares that `centers` came from
    get_aabb_2d(means, scales, glob_scale, quats, viewmat, (fx, fy, cx, cy)): the backward then chains the centre
    gradient through the AABB itself (gstex_raster_setup_bwd_aabb) and returns none for `centers`, so neither
    get_aabb_2d's backward nor autograd's accumulation kernels run.  Same gradients, bit for bit.

    geometry_outputs=False (not in the reference API): depth, reg and normal are not produced (returned as
    zeros without gradient) -- the photometric training step, whose loss does not read them (gstex.py:1313-1317
    with the default zero normal / distortion weights); the other outputs are unchanged.

    texture_grad_sink (not in the reference API; multi-GPU training): a zeroed contiguous fp32 tensor shaped like
    `texture` that the backward accumulates the texel gradient into (e.g. the texel slice of a flat all-reduce
    buffer); autograd then receives no gradient for `texture`, and on_texture_grad() (if given) is called once the
    kernel producing it has been enqueued.  zero_texture_grad_sink=True: the raster forward zeroes the sink itself
    (the first render of a step; leave it False for the renders whose gradients accumulate on top).

    texture_ready (not in the reference API): a torch.cuda.Event the current stream waits on right before the raster
    forward -- the texel update of the previous optimizer step running on a side stream (GStexTrainer
    async_texture), so preprocessing and binning overlap it -- or a callable run at that point (GStexTrainer
    defer_texture under GradSync: the deferred texel update, which first waits for its collective).

    before_pair_wait (not in the reference API): a callable run after the pair-count read-back has been queued and
    before the host waits for it -- work it enqueues keeps the device busy through that wait (GStexTrainer
    defer_texture: the previous step's texel update).

    pair_guard (not in the reference API; training loops): (PairCapacity, step_flag, first, tag) -- capacity mode: the
    pair buffers are sized from the PairCapacity and the pair total stays on the device (no read-back, no wait); the
    render's guard writes 1.0 into step_flag (a 1-element device fp32 view; first=True overwrites it, else the larger
    value is kept) when the total exceeds the capacity, in which case every output is the empty render's and the
    optimizer step guarded by that flag does nothing (FusedAdam.step(skip_flag=...)).

    binning (not in the reference API): a Binning from bin_gaussians() on the same centers / extents / depths /
    num_tiles_hit tensors -- several renders of one geometry (the eval render's three calls, gstex.py:1165-1200)
    bin and sort once.

    Returns (img (H,W,3), depth (H,W), reg (H,W), alpha (H,W), tex_img (H,W,C), normal (H,W,3)).
    Gradients flow to rgbs, opacities, means, scales, quats, texture, centers (-> get_aabb_2d),
    uv0 and background; umap/vmap are treated as constants (detached by the caller, gstex.py:977-984).
    """
    if use_torch_impl:
        raise NotImplementedError(
            "texture_gaussians(use_torch_impl=True): gstex_amd ships no CPU rasterizer; "
            "the CPU restatement in oracle/ is test infrastructure only")
    return _TextureGaussians.apply(texture_info, texture_dims, centers, extents, depths, num_tiles_hit, rgbs,
                                   opacities, means, scales, glob_scale, quats, uv0, umap, vmap, texture, viewmat,
                                   c2w, fx, fy, cx, cy, H, W, block_width, settings, background, texture_transform,
                                   fold_aabb, geometry_outputs, torch.is_grad_enabled(), texture_grad_sink,
                                   on_texture_grad, texture_ready, binning, before_pair_wait, zero_texture_grad_sink,
                                   pair_guard)


class Binning(NamedTuple):
    """bin_gaussians() output, reusable by texture_gaussians(binning=...) calls on the same geometry."""
    n: int
    H: int
    W: int
    nth: torch.Tensor
    offsets: torch.Tensor
    tile_ranges: torch.Tensor
    sorted_ids: torch.Tensor
    sorted_slots: torch.Tensor
    order: torch.Tensor


def bin_gaussians(centers, extents, depths, num_tiles_hit, H: int, W: int) -> Binning:
    """Tile binning + depth sort + largest-first tile order of one geometry, for several texture_gaussians calls."""
    n = centers.shape[0]
    nth = _i32(num_tiles_hit, "num_tiles_hit", (n,))
    c = _f32(centers.detach(), "centers", (n, 2))
    e = _f32(extents.detach(), "extents", (n, 2))
    d = _f32(depths.detach(), "depths", (n,))
    out = bin_finish(bin_begin(nth), c, e, d, int(H), int(W), BLOCK_WIDTH, with_order=True)
    return Binning(n, int(H), int(W), nth, *out)


rasterize_gaussians = texture_gaussians  # north_star name


# ----------------------------------------------------------------------------------------
# spherical harmonics
# ----------------------------------------------------------------------------------------
def num_sh_bases(degree: int) -> int:
    """(degree+1)^2 (gstex.py:307)."""
    if degree < 0 or degree > 4:
        raise ValueError(f"SH degree must be in [0, 4] (got {degree})")
    return (degree + 1) ** 2


class _SH(torch.autograd.Function):
    @staticmethod
    def forward(ctx, degree, viewdirs, coeffs):
        viewdirs = _f32(viewdirs.detach(), "viewdirs", (None, 3))
        n = viewdirs.shape[0]
        coeffs = _f32(coeffs, "coeffs", (n, None, 3))
        K = coeffs.shape[1]
        _check(K >= num_sh_bases(degree), f"coeffs has {K} bases < (degree+1)^2 = {num_sh_bases(degree)}")
        out = torch.empty((n, 3), device=coeffs.device, dtype=torch.float32)
        call("gstex_sh_fwd", n, int(degree), K, ptr(viewdirs), ptr(coeffs), ptr(out), _stream(coeffs))
        ctx.save_for_backward(viewdirs)
        ctx.degree, ctx.K = int(degree), K
        return out

    @staticmethod
    def backward(ctx, v_out):
        (viewdirs,) = ctx.saved_tensors
        n = viewdirs.shape[0]
        v_coeffs = torch.empty((n, ctx.K, 3), device=viewdirs.device, dtype=torch.float32)
        call("gstex_sh_bwd", n, ctx.degree, ctx.K, ptr(viewdirs), ptr(v_out.contiguous()), ptr(v_coeffs),
             _stream(viewdirs))
        return None, None, v_coeffs


def spherical_harmonics(degrees_to_use: int, viewdirs: torch.Tensor, coeffs: torch.Tensor) -> torch.Tensor:
    """View-dependent colour sum_k basis_k(dir) coeffs[:, k] (no +0.5, gstex.py:1099-1114).
    Differentiable w.r.t. coeffs only (the caller detaches viewdirs)."""
    return _SH.apply(int(degrees_to_use), viewdirs, coeffs)


# ----------------------------------------------------------------------------------------
# texture_sample
# ----------------------------------------------------------------------------------------
class _TextureSample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, C, query_dims, texture, uv):
        qd = _i32(query_dims, "query_dims", (None, 3))
        nq = qd.shape[0]
        texture = _f32(texture, "texture", (None, C))
        uv = _f32(uv.detach(), "uv", (nq, 2))
        out = torch.empty((nq, C), device=texture.device, dtype=torch.float32)
        call("gstex_texture_sample", nq, C, ptr(qd), ptr(texture), texture.shape[0], ptr(uv), ptr(out),
             _stream(texture))
        ctx.save_for_backward(qd, uv)
        ctx.C, ctx.T = C, texture.shape[0]
        return out

    @staticmethod
    def backward(ctx, v_out):
        qd, uv = ctx.saved_tensors
        v_tex = torch.zeros((ctx.T, ctx.C), device=qd.device, dtype=torch.float32)
        call("gstex_texture_sample_bwd", qd.shape[0], ctx.C, ptr(qd), ctx.T, ptr(uv), ptr(v_out.contiguous()),
             ptr(v_tex), _stream(qd))
        return None, None, v_tex, None


def texture_sample(texture_info, query_dims, texture, uv, use_torch_impl=False):
    """Resample jagged textures at per-texel UVs (jagged_texture.py:135-138) -> (T', C).
    use_torch_impl=True runs the reference-API pure-torch sampler gstex_cuda._torch_impl.sample_texture."""
    C = int(texture_info[-1])
    if use_torch_impl:
        from gstex_cuda._torch_impl import sample_texture

        return sample_texture(query_dims, texture, uv)
    return _TextureSample.apply(C, query_dims, texture, uv)


@torch.no_grad()
def texture_edit(texture_info, texture_dims, edit_rgb, edit_alpha, depth_lower, depth_upper, centers, extents, depths,
                 num_tiles_hit, opacities, means, scales, glob_scale, quats, uv0, umap, vmap, viewmat, c2w, fx, fy,
                 cx, cy, H, W, block_width, settings, background=None, use_torch_impl=False):
    """gstex_cuda.texture_edit.texture_edit (gstex.py:579-600): back-project a screen-space RGBA stroke
    onto the texels.  Returns (T, 5) = per texel sum of  b * w * (a*rgb, a, 1)  over the pixel-splat
    pairs whose hit depth lies in [depth_lower, depth_upper] (b: bilinear weight, w = alpha * T, a: the
    stroke alpha); the caller forms colour = out[:, :3] / out[:, 3] and weight = out[:, 3] / out[:, 4]
    (gstex.py:602-605).  texture_info = (N, 1, 5)."""
    if use_torch_impl:
        raise NotImplementedError("texture_edit(use_torch_impl=True): gstex_amd has no CPU rasterizer")
    N, L, K = (int(v) for v in texture_info)
    _check(L == 1 and K == 5, f"texture_info must be (N, 1, 5) for texture_edit (got {tuple(texture_info)})")
    _check(int(block_width) == BLOCK_WIDTH, f"block_width must be {BLOCK_WIDTH} (got {block_width})")
    means = _f32(means, "means", (None, 3))
    n = means.shape[0]
    _check(N == n, f"texture_info[0] ({N}) != number of splats ({n})")
    H, W = int(H), int(W)
    dims = _i32(texture_dims, "texture_dims", (n, 3))
    centers_c = _f32(centers, "centers", (n, 2))
    extents_c = _f32(extents, "extents", (n, 2))
    depths_c = _f32(depths, "depths", (n,))
    nth = _i32(num_tiles_hit, "num_tiles_hit", (n,))
    opacities = _f32(opacities, "opacities", (n, 1))
    scales = _f32(scales, "scales", (n, 3))
    quats = _f32(quats, "quats", (n, 4))
    uv0 = _f32(uv0, "uv0", (n, 1, 2))
    umap = _f32(umap, "umap", (n, 1, 3))
    vmap = _f32(vmap, "vmap", (n, 1, 3))
    rgb = _f32(edit_rgb, "edit_rgb", (H, W, 3))
    a = _f32(edit_alpha.reshape(H, W), "edit_alpha", (H, W))
    dlo = _f32(depth_lower, "depth_lower", (H, W))
    dhi = _f32(depth_upper, "depth_upper", (H, W))
    vm = _viewmat(viewmat)
    cw = _c2w(c2w)
    dev = means.device
    st = _stream(means)
    cam = _lib.make_camera(vm, cw, fx, fy, cx, cy, H, W, BLOCK_WIDTH)
    n_texels = int((dims[:, 0].long() * dims[:, 1].long()).sum()) if n else 0
    if n:
        n_texels = max(n_texels, int((dims[:, 2].long() + dims[:, 0].long() * dims[:, 1].long()).max()))
    out = torch.zeros((n_texels, 5), device=dev, dtype=torch.float32)
    offsets, tile_ranges, sorted_ids, _ = bin_and_sort(centers_c, extents_c, depths_c, nth, H, W, BLOCK_WIDTH)
    order = tile_order(tile_ranges)
    records = torch.empty((n, REC_FLOATS), device=dev, dtype=torch.float32)
    zeros3 = torch.zeros((n, 3), device=dev, dtype=torch.float32)  # colours do not enter the edit
    _launch("gstex_raster_setup", n, ptr(means), ptr(scales), float(glob_scale), ptr(quats), ptr(zeros3),
            ptr(opacities), ptr(centers_c), ptr(uv0), ptr(umap), ptr(vmap), ptr(dims), ptr(nth), cam, ptr(records), None,
            st)
    _launch("gstex_texture_edit", cam, int(settings), ptr(records), ptr(tile_ranges), ptr(order), ptr(sorted_ids),
            ptr(rgb), ptr(a), ptr(dlo), ptr(dhi), n_texels, ptr(out), st)
    return out
