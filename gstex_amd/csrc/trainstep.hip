// trainstep.hip — host-side sequencing of a photometric training render's launches before its raster forward
// (gstex_train_prologue, ABI 17; gstex_amd.fused).  Each call below is the per-op C-ABI entry point with the
// arguments gstex_amd's per-op Python path passes it, so the device work is identical; what goes away is the host
// time between the launches (Python, ctypes, autograd nodes, allocations), which a step starting on an idle device
// (the first one after a synchronisation) otherwise spends with the device waiting.
#include "gstex_common.h"
#include "gstex_error.h"

extern "C" int gstex_train_prologue(const gstex_train_prologue_args* a, void* stream) {
    GSTEX_REQUIRE(a, "gstex_train_prologue: null arguments");
    GSTEX_REQUIRE(a->n >= 0 && a->capacity >= 0, "gstex_train_prologue: invalid sizes (n %d)", a->n);
    int rc = gstex_activate_fwd(a->n, a->means, a->quats, a->log_scales, a->opac_logits, a->mappings, a->map_cols,
                                a->campos, a->quats_n, a->scales, a->opacities, a->uv0, a->umap, a->vmap,
                                a->viewdirs, stream);
    if (rc) return rc;
    gstex_camera pre = a->cam;  // preprocessing takes the view without c2w (as gstex_amd.ops.preprocess)
    pre.c2w = nullptr;
    rc = gstex_preprocess(a->n, a->means, a->scales, 1.0f, a->quats_n, &pre, a->depths, a->centers, a->extents,
                          a->num_tiles_hit, stream);
    if (rc) return rc;
    rc = gstex_sh_rest_fwd(a->n, a->sh_degree, a->n_rest, a->viewdirs, a->features_rest, a->rgbs, stream);
    if (rc) return rc;
    rc = gstex_scan_offsets_guarded(a->n, a->num_tiles_hit, a->offsets, a->scan_workspace, a->scan_workspace_bytes,
                                    &a->guard, stream);
    if (rc) return rc;
    rc = gstex_raster_setup(a->n, a->means, a->scales, 1.0f, a->quats_n, a->rgbs, a->opacities, a->centers, a->uv0,
                            a->umap, a->vmap, a->texture_dims, a->num_tiles_hit, &a->cam, a->records, stream);
    if (rc) return rc;
    return gstex_bin_sort_capped(a->n, a->capacity, a->centers, a->extents, a->depths, a->num_tiles_hit, a->offsets,
                                 a->cam.H, a->cam.W, a->cam.block, a->tile_ranges, a->sorted_ids, a->sorted_slots,
                                 a->tile_order, a->bin_workspace, a->bin_workspace_bytes, stream);
}
