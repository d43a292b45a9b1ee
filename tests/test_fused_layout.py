"""Host logic of gstex_amd.fused (no GPU): the arena layout of the fused training render -- every buffer 256-byte
aligned, no two overlapping, each as large as the C-ABI size queries ask (scan / bin workspaces, raster aux) -- and
the gradient arena's 256-byte-aligned slices."""
import pytest

from gstex_amd import _lib, fused


@pytest.mark.parametrize("n,n_rest,cap,H,W", [(1, 15, 1, 16, 16), (300, 15, 10_000, 96, 96),
                                              (200_000, 15, 2_930_000, 800, 800), (4097, 3, 70_000, 100, 130)])
def test_arena_layout(n, n_rest, cap, H, W):
    lib = _lib.load()
    off, total, sizes, goff, gfloats = fused._layout(n, n_rest, cap, H, W, 3)
    n_tiles = ((W + 15) // 16) * ((H + 15) // 16)
    assert sizes["n_tiles"] == n_tiles
    assert sizes["scan_ws"] >= lib.gstex_train_prologue_scan_bytes(n)
    assert sizes["bin_ws"] >= lib.gstex_bin_workspace_size(n, cap, n_tiles)
    assert sizes["aux"] == lib.gstex_raster_aux_bytes(cap, n_tiles, 3)
    need = {"quats_n": 16 * n, "records": 4 * _lib.REC_FLOATS * n, "sorted_ids": 4 * cap, "sorted_slots": 4 * cap,
            "tile_ranges": 8 * n_tiles, "img": 12 * H * W, "state": 16 * H * W, "partials": 4 * _lib.PARTIAL_FLOATS * n,
            "scan_ws": sizes["scan_ws"], "bin_ws": sizes["bin_ws"], "aux": sizes["aux"], "offsets": 4 * (n + 1)}
    order = sorted(off.items(), key=lambda kv: kv[1])
    for (name, o), (_, nxt) in zip(order, order[1:] + [("end", total)]):
        assert o % 256 == 0, name
        if name in need:
            assert nxt - o >= need[name], f"{name}: {nxt - o} bytes < {need[name]}"
        assert nxt > o or (name == order[-1][0] and nxt >= o)
    g = sorted(goff.items(), key=lambda kv: kv[1])
    per = {"means": 3 * n, "quats": 4 * n, "log_scales": 3 * n, "opac_logits": n, "features_rest": 3 * n_rest * n}
    for (name, o), (_, nxt) in zip(g, g[1:] + [("end", gfloats)]):
        assert o % 64 == 0 and nxt - o >= per[name], name
