"""The photometric training render as one autograd node (not in the reference; GStexTrainer(fused_step=True)).

GStexTrainer.render's training branch (gstex.py:992-1162 with the fused activations, the zeroed SH DC term and the
read-back-free pair buffers) issues eight C calls before its raster forward -- activate, preprocess, sh_rest, the
guarded scan (three kernels), the splat records, the capped binning -- each behind its own Python wrapper, ctypes
call, autograd node and a dozen tensor allocations.  Here they are one C call (gstex_train_prologue, ABI 17) into one
arena allocation: activate + preprocess + sh_rest as one per-splat kernel and the scan as one launch (the same device
functions on the same values, gstex_amd/csrc/splat_math.h: bit-identical outputs), then the records and the binning
as before; the backward is the raster backward and one epilogue call (gstex_train_epilogue: setup bwd, SH rest bwd
and activation bwd as one per-splat kernel, again on shared device functions).
tests/test_gpu_fused.py compares both paths.  What it removes is host time between the launches, which the device
waits through whenever a step starts on an idle device -- the first step after a synchronisation (bench.py's first
timed step) -- and four launches.

Taken only where it applies (GStexTrainer._fused_ok): a texel-gradient sink (defer_texture, or GradSync's flat buffer
at N > 1: its route, tail-collective callback and late texel update are honoured as in the per-op render), a sized
PairCapacity, SH degree > 0 without fix_init, no geometry outputs, non-deterministic accumulation, not capturing.
Every other case runs the per-op path unchanged.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib, ops
from ._lib import PARTIAL_FLOATS, REC_FLOATS, ptr
from .charts import SH_C0  # SH2RGB(texture_dc) applied by the raster on read (gstex.py:1119), as GStexTrainer.render

_ALIGN = 256
_LAYOUTS: dict = {}


def _layout(n: int, n_rest: int, capacity: int, H: int, W: int, C: int):
    """Byte offsets of the render's buffers in one arena, and the final gradients' offsets in a second one."""
    key = (n, n_rest, capacity, H, W, C)
    hit = _LAYOUTS.get(key)
    if hit is not None:
        return hit
    lib = _lib.load()
    n_tiles = ((W + ops.BLOCK_WIDTH - 1) // ops.BLOCK_WIDTH) * ((H + ops.BLOCK_WIDTH - 1) // ops.BLOCK_WIDTH)
    f4 = 4
    scan_ws = max(int(lib.gstex_train_prologue_scan_bytes(n)), 1)
    bin_ws = max(int(lib.gstex_bin_workspace_size(n, capacity, n_tiles)), 1)
    aux = int(lib.gstex_raster_aux_bytes(capacity, n_tiles, C))
    items = [  # forward: the prologue's outputs, the raster's outputs and its record for the backward
        ("quats_n", 4 * n * f4), ("scales", 3 * n * f4), ("opacities", n * f4), ("uv0", 2 * n * f4),
        ("umap", 3 * n * f4), ("vmap", 3 * n * f4), ("viewdirs", 3 * n * f4), ("depths", n * f4),
        ("centers", 2 * n * f4), ("extents", 2 * n * f4), ("num_tiles_hit", n * 4), ("rgbs", 3 * n * f4),
        ("offsets", (n + 1) * 4), ("scan_ws", scan_ws), ("records", REC_FLOATS * n * f4),
        ("hp", _lib.HP_DOUBLES * n * 8),
        ("tile_ranges", 2 * n_tiles * 4), ("sorted_ids", capacity * 4), ("sorted_slots", capacity * 4),
        ("tile_order", n_tiles * 4), ("bin_ws", bin_ws),
        ("img", 3 * H * W * f4), ("alpha", H * W * f4), ("tex", C * H * W * f4), ("state", 4 * H * W * f4),
        ("aux", max(aux, 1)), ("partials", PARTIAL_FLOATS * n * f4),
        # backward intermediates (the activated parameters' gradients)
        ("v_scales", 3 * n * f4), ("v_quats_n", 4 * n * f4), ("v_rgbs", 3 * n * f4), ("v_opacities", n * f4),
        ("v_centers", 2 * n * f4), ("v_uv0", 2 * n * f4)]
    off, pos = {}, 0
    for name, nb in items:
        off[name] = pos
        pos += (nb + _ALIGN - 1) // _ALIGN * _ALIGN
    grads = [("means", 3 * n), ("quats", 4 * n), ("log_scales", 3 * n), ("opac_logits", n),
             ("features_rest", 3 * n_rest * n)]
    goff, gpos = {}, 0
    for name, nf in grads:
        goff[name] = gpos
        gpos += (nf + 63) // 64 * 64  # floats (256-byte aligned)
    hit = (off, pos, dict(aux=aux, scan_ws=scan_ws, bin_ws=bin_ws, n_tiles=n_tiles), goff, gpos)
    if len(_LAYOUTS) >= 64:  # (the capacity grows and recharts change n: keep the cache bounded)
        _LAYOUTS.clear()
    _LAYOUTS[key] = hit
    return hit


def _view(arena: torch.Tensor, off: int, shape) -> torch.Tensor:
    """fp32 view of arena bytes [off, off + 4 * prod(shape))."""
    nb = 4
    for s in shape:
        nb *= s
    return arena[off:off + nb].view(torch.float32).view(shape)


class _TrainRender(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tr, view, degree, sink, zero_sink, first, on_grad, texture_ready, zero_next, means, quats,
                log_scales, opac_logits, features_rest):
        n = means.shape[0]
        n_rest = features_rest.shape[1]
        H, W, C = int(view.H), int(view.W), 3
        dev = means.device
        st = _lib.stream_of(dev)
        pcap = tr.pairs
        step_flag = tr._skip_flag()
        # `first`: the step's first render, which resets the step's guard flag (not whether the sink is zeroed here:
        # with the double-buffered texel gradient the previous backward zeroed it)
        guard, slot, cap = pcap.reserve(step_flag, bool(first), tr.step)
        off, nbytes, sizes, goff, gfloats = _layout(n, n_rest, cap, H, W, C)
        arena = torch.empty((nbytes,), device=dev, dtype=torch.uint8)
        base = arena.data_ptr()
        P = {k: base + v for k, v in off.items()}
        vm = ops._viewmat(view.viewmat)
        cw = ops._c2w(view.c2w)
        cam = _lib.make_camera(vm, cw, view.fx, view.fy, view.cx, view.cy, H, W, ops.BLOCK_WIDTH)
        mp = tr.mappings
        a = _lib.GstexTrainPrologueArgs(
            n=n, sh_degree=int(degree), n_rest=n_rest, map_cols=mp.shape[1], capacity=cap, cam=cam, guard=guard,
            means=ptr(means), quats=ptr(quats), log_scales=ptr(log_scales), opac_logits=ptr(opac_logits),
            mappings=ptr(mp), campos=ptr(view.campos), features_rest=ptr(features_rest),
            texture_dims=ptr(tr.texture_dims),
            quats_n=P["quats_n"], scales=P["scales"], opacities=P["opacities"], uv0=P["uv0"], umap=P["umap"],
            vmap=P["vmap"], viewdirs=P["viewdirs"], depths=P["depths"], centers=P["centers"], extents=P["extents"],
            num_tiles_hit=P["num_tiles_hit"], rgbs=P["rgbs"], offsets=P["offsets"], scan_workspace=P["scan_ws"],
            scan_workspace_bytes=sizes["scan_ws"], records=P["records"], tile_ranges=P["tile_ranges"],
            sorted_ids=P["sorted_ids"], sorted_slots=P["sorted_slots"], tile_order=P["tile_order"],
            bin_workspace=P["bin_ws"], bin_workspace_bytes=sizes["bin_ws"],
            raster_aux=P["aux"] if sizes["aux"] else None, raster_aux_bytes=sizes["aux"], raster_channels=C,
            hp_records=P["hp"] if ops.HP_RECORDS else None)
        _lib.call("gstex_train_prologue", ctypes.byref(a), st)
        pcap.commit(slot, cap, tr.step, dev)
        if texture_ready is not None:  # the deferred texel update waiting for its collective: the raster forward
            texture_ready()            # is the first reader of the texels
        texture = tr.texture_dc
        zn = sink.numel() if zero_sink else 0
        aux_zeroed = _lib.SETTING_AUX_ZEROED if sizes["aux"] else 0  # (zeroed by the prologue's scan kernel)
        ops._launch("gstex_raster_fwd_zero", cam, C, int(tr.settings) | aux_zeroed, ptr(tr._bg_zero), P["records"],
                    P["hp"] if ops.HP_RECORDS else None, P["tile_ranges"], P["tile_order"], P["sorted_ids"], ptr(texture), texture.shape[0],
                    SH_C0, 0.5, P["img"], None, None, P["alpha"], P["tex"], None, P["state"], cap,
                    P["aux"] if sizes["aux"] else None, ptr(sink) if zero_sink else None, zn, P["partials"],
                    PARTIAL_FLOATS * n, st)
        ctx.tr, ctx.arena, ctx.P, ctx.cam_keep = tr, arena, P, (vm, cw)
        ctx.cam, ctx.cap, ctx.sink, ctx.degree, ctx.goff, ctx.gfloats = cam, cap, sink, int(degree), goff, gfloats
        ctx.on_grad = on_grad
        ctx.zero_next = zero_next
        ctx.has_aux = sizes["aux"] > 0
        ctx.save_for_backward(quats, log_scales)
        ctx.set_materialize_grads(False)
        img = _view(arena, off["img"], (H, W, 3))
        alpha = _view(arena, off["alpha"], (H, W))
        tex = _view(arena, off["tex"], (H, W, C))
        return img, alpha, tex

    @staticmethod
    def backward(ctx, v_img, v_alpha, v_tex):
        quats, log_scales = ctx.saved_tensors
        tr, P, cam = ctx.tr, ctx.P, ctx.cam
        n = quats.shape[0]
        dev = quats.device
        st = _lib.stream_of(dev)
        c = lambda t: None if t is None else t.contiguous()  # noqa: E731
        v_img, v_alpha, v_tex = c(v_img), c(v_alpha), c(v_tex)
        texture = tr.texture_dc
        bwd_args = (cam, 3, int(tr.settings), ptr(tr._bg_zero),
                    P["records"], P["hp"] if ops.HP_RECORDS else None, P["tile_ranges"], P["sorted_ids"], P["sorted_slots"], ptr(texture),
                    texture.shape[0], SH_C0, 0.5, P["state"], ptr(v_img), None, None, ptr(v_alpha), ptr(v_tex), None,
                    ctx.cap, P["partials"], None, ptr(ctx.sink), P["aux"] if ctx.has_aux else None)
        zn = ctx.zero_next
        if zn is not None and zn is tr._tex_grad_next and zn.data_ptr() != ctx.sink.data_ptr():
            # the trainer's other texel-gradient buffer, zeroed by this backward's grid for the next step
            ops._launch("gstex_raster_bwd_zero", *bwd_args, ptr(zn), zn.numel(), st)
            tr._next_zeroed = True
        else:
            ops._launch("gstex_raster_bwd", *bwd_args, st)
        ctx.zero_next = None
        if ctx.on_grad is not None:
            ctx.on_grad()  # the texel gradient is complete in stream order (GradSync starts its tail collective)
        grads = torch.empty((ctx.gfloats,), device=dev, dtype=torch.float32)
        g = {k: grads.data_ptr() + 4 * v for k, v in ctx.goff.items()}
        means = tr.means
        n_rest = tr.features_rest.shape[1]
        # setup bwd -> activations bwd + SH rest bwd in one launch (gstex_train_epilogue)
        e = _lib.GstexTrainEpilogueArgs(
            n=n, sh_degree=ctx.degree, n_rest=n_rest, cam=cam, means=ptr(means), scales=P["scales"],
            quats_n=P["quats_n"], quats=ptr(quats), log_scales=ptr(log_scales), opacities=P["opacities"],
            umap=P["umap"], vmap=P["vmap"], viewdirs=P["viewdirs"], num_tiles_hit=P["num_tiles_hit"],
            offsets=P["offsets"], partials=P["partials"], v_means=g["means"], v_quats=g["quats"],
            v_log_scales=g["log_scales"], v_opac_logits=g["opac_logits"], v_features_rest=g["features_rest"],
            v_scales_act=P["v_scales"], v_quats_n=P["v_quats_n"], v_rgbs=P["v_rgbs"], v_opacities_act=P["v_opacities"],
            v_centers=P["v_centers"], v_uv0=P["v_uv0"])
        _lib.call("gstex_train_epilogue", ctypes.byref(e), st)
        ctx.arena = None
        o = ctx.goff

        def gv(name, shape):
            return _view_f(grads, o[name], shape)
        return (None, None, None, None, None, None, None, None, None, gv("means", (n, 3)), gv("quats", (n, 4)), gv("log_scales", (n, 3)),
                gv("opac_logits", (n, 1)), gv("features_rest", (n, n_rest, 3)))


def _view_f(flat: torch.Tensor, off: int, shape) -> torch.Tensor:
    nf = 1
    for s in shape:
        nf *= s
    return flat[off:off + nf].view(shape)


def train_render(tr, view, degree: int, sink: torch.Tensor, zero_sink: bool, first: bool, on_grad=None,
                 texture_ready=None, zero_next=None):
    """-> (img (H,W,3), alpha (H,W), tex (H,W,3)) of GStexTrainer.render's photometric training branch; the texel
    gradient accumulates into `sink` (zeroed by the raster forward when zero_sink), `first` marks the step's first
    render (it resets the step's pair-capacity guard flag), and on_grad() runs once the raster
    backward is enqueued; texture_ready() (a deferred texel update) runs right before the raster forward; zero_next
    (the trainer's other texel-gradient buffer) is zeroed by the raster backward's grid."""
    return _TrainRender.apply(tr, view, degree, sink, zero_sink, first, on_grad, texture_ready, zero_next, tr.means,
                              tr.quats, tr.scales, tr.opacities, tr.features_rest)
