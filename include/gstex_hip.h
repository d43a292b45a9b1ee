/*
 * gstex_hip.h — C-ABI of libgstex_hip.so, the MI355X (gfx950) textured-2DGS rasterizer.
 *
 * This is the drop-in boundary for the `gstex_cuda` native extension that the reference
 * (nvnhat95/GStex) imports but does not vendor (`.gitmodules:1-3`, submodules/GStex_cuda is
 * empty).  Each entry point below replaces one native op behind a reference call site:
 *
 *   gstex_project_points      <- gstex_cuda.get_aabb_2d.project_points      (nerfstudio/models/gstex.py:1077)
 *   gstex_aabb_2d(+_bwd)      <- gstex_cuda.get_aabb_2d.get_aabb_2d          (gstex.py:1079)
 *   gstex_num_tiles_hit       <- gstex_cuda.get_aabb_2d.get_num_tiles_hit_2d (gstex.py:1080)
 *   gstex_scan_offsets,
 *   gstex_bin_sort            <- tile binning + per-tile depth sort inside texture_gaussians
 *                                (args gstex.py:1136-1139,1158)
 *   gstex_raster_setup,
 *   gstex_raster_fwd          <- gstex_cuda.texture.texture_gaussians forward (gstex.py:1133-1162)
 *   gstex_raster_bwd,
 *   gstex_raster_setup_bwd    <- texture_gaussians backward (autograd, engine/trainer.py:460)
 *   gstex_sh_fwd / _bwd       <- gstex_cuda.sh.spherical_harmonics           (gstex.py:1109,1111)
 *   gstex_texture_sample(+_bwd) <- gstex_cuda.texture_sample.texture_sample  (models/jagged_texture.py:138)
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer to contiguous row-major fp32 / int32 memory, except
 *     `const gstex_camera*` which is a HOST struct (read at call time) of device pointers.
 *   - `stream` is a hipStream_t (NULL = default stream). Calls only enqueue work: no allocation,
 *     no host synchronisation.
 *   - Scratch memory is caller-owned: query the size with the *_workspace_size function, allocate
 *     it (e.g. with the torch caching allocator) and pass it in.
 *   - Return value: 0 (GSTEX_OK) or a gstex_status; the message of the last failure on the calling
 *     thread is returned by gstex_last_error().
 */
#ifndef GSTEX_HIP_H
#define GSTEX_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 18 (round 6): the hipGraph step support of ABI 16 (event-record nodes, gstex_adam_step_scheduled) and the
 * split-backward settings bit of ABI 15 are removed (measured slower). */
#define GSTEX_ABI_VERSION 18

/* Per-record layout of the splat table written by gstex_raster_setup (floats). */
#define GSTEX_REC_FLOATS 32
/* Per-(tile, splat, quadrant) gradient partial row written by gstex_raster_bwd (floats). */
#define GSTEX_PARTIAL_FLOATS 32
#define GSTEX_PARTIAL_FLOATS_PHOTO 24
/* Per-splat fp64 row of a near-edge-on splat written by gstex_raster_setup into hp_records (doubles, ABI 18). */
#define GSTEX_HP_DOUBLES 12

/* settings bitfield (GStexModelConfig.settings, gstex.py:194-197) */
#define GSTEX_SETTING_AA_BLUR (1 << 9)   /* 2DGS screen-space low-pass */
#define GSTEX_SETTING_DIST_REG (1 << 10) /* 2DGS NDC depth-distortion output */
#define GSTEX_SETTING_EDIT (1 << 13)     /* texture_edit request (gstex.py:599) */
#define GSTEX_SETTING_EVAL_NORMAL (1 << 15) /* eval normal/edit render (gstex.py:1198): normal output unit-length, forward only */
/* gstex_raster_fwd / gstex_raster_fwd_zero only (ABI 17): the aux span the forward accumulates its unit costs, launch
 * order and unit-order histogram into was zeroed by gstex_train_prologue (args.raster_aux, same n_isect / tiles /
 * channels) on the same stream, so the forward skips its own fill.  Set it only after such a prologue call. */
#define GSTEX_SETTING_AUX_ZEROED (1 << 28)

typedef enum {
    GSTEX_OK = 0,
    GSTEX_ERR_INVALID_ARG = 1,
    GSTEX_ERR_LAUNCH = 2,
    GSTEX_ERR_UNSUPPORTED = 3,
    GSTEX_ERR_WORKSPACE = 4
} gstex_status;

/* Pinhole camera (a HOST struct holding DEVICE pointers, so no host sync is needed to read the
 * model's on-GPU matrices).  viewmat = first 3 rows of world->camera (OpenCV axes, after the y/z
 * flip of gstex.py:1031-1041), row-major DEVICE float[12].  c2w = its inverse, row-major DEVICE
 * float[16] (only the camera centre c2w[:3,3] is read; NULL = derive it from viewmat). */
typedef struct {
    const float* viewmat;
    const float* c2w;
    float fx, fy, cx, cy;
    int32_t H, W, block;
} gstex_camera;

const char* gstex_last_error(void);
int gstex_abi_version(void);

/* ---- per-splat preprocessing ---------------------------------------------------------- */
int gstex_project_points(int32_t n, const float* means, const gstex_camera* cam,
                         float* xys, float* depths, void* stream);
int gstex_project_points_bwd(int32_t n, const float* means, const gstex_camera* cam,
                             const float* v_xys, const float* v_depths, float* v_means,
                             void* stream);
int gstex_aabb_2d(int32_t n, const float* means, const float* scales, float glob_scale,
                  const float* quats, const gstex_camera* cam, float* centers, float* extents,
                  void* stream);
/* Writes the gradient of the AABB centre to v_means / v_scales / v_quats (every element; zero for
   splats with no centre gradient or culled). */
int gstex_aabb_2d_bwd(int32_t n, const float* means, const float* scales, float glob_scale,
                      const float* quats, const gstex_camera* cam, const float* v_centers,
                      float* v_means, float* v_scales, float* v_quats, void* stream);
int gstex_num_tiles_hit(int32_t n, const float* centers, const float* extents, int32_t H,
                        int32_t W, int32_t block, int32_t* num_tiles_hit, void* stream);
/* The three preprocessing outputs a render needs, in one pass (ABI 10): depths[n] (the view depth of
 * gstex_project_points), centers / extents[n][2] (gstex_aabb_2d) and num_tiles_hit[n]
 * (gstex_num_tiles_hit with cam->H, cam->W, cam->block), bit-identical to the three calls.  No
 * backward: a caller that needs the centre gradient uses gstex_raster_setup_bwd_aabb (fold). */
int gstex_preprocess(int32_t n, const float* means, const float* scales, float glob_scale,
                     const float* quats, const gstex_camera* cam, float* depths, float* centers,
                     float* extents, int32_t* num_tiles_hit, void* stream);

/* ---- binning + per-tile depth sort ---------------------------------------------------- */
size_t gstex_scan_workspace_size(int32_t n);
/* offsets[0..n] = exclusive prefix sum of num_tiles_hit; offsets[n] = total intersections. */
int gstex_scan_offsets(int32_t n, const int32_t* num_tiles_hit, int32_t* offsets,
                       void* workspace, size_t workspace_bytes, void* stream);
size_t gstex_bin_workspace_size(int32_t n, int64_t n_isect, int32_t n_tiles);
/* Emits one (tile, splat) pair per covered tile, buckets them per tile and sorts every tile's
 * list by (depth bits, splat id).  Outputs: tile_ranges[n_tiles][2] = [start, end) into
 * sorted_ids; sorted_ids[n_isect] = splat id; sorted_slots[n_isect] = emission index
 * offsets[id] + k (k = row-major rank of the tile inside the splat's tile rectangle). */
int gstex_bin_sort(int32_t n, int64_t n_isect, const float* centers, const float* extents,
                   const float* depths, const int32_t* num_tiles_hit, const int32_t* offsets,
                   int32_t H, int32_t W, int32_t block, int32_t* tile_ranges,
                   int32_t* sorted_ids, int32_t* sorted_slots, void* workspace,
                   size_t workspace_bytes, void* stream);
/* gstex_bin_sort that also writes tile_order[n_tiles] (non-NULL), the largest-first launch order
 * gstex_tile_order would compute from the resulting tile_ranges (same keys, same ranking): the
 * tile sort already ranks the buckets, so the raster forward reuses that order instead of a
 * second ranking launch.  ABI 8. */
int gstex_bin_sort_ordered(int32_t n, int64_t n_isect, const float* centers, const float* extents,
                           const float* depths, const int32_t* num_tiles_hit, const int32_t* offsets,
                           int32_t H, int32_t W, int32_t block, int32_t* tile_ranges,
                           int32_t* sorted_ids, int32_t* sorted_slots, int32_t* tile_order,
                           void* workspace, size_t workspace_bytes, void* stream);

/* ---- read-back-free binning (ABI 13) -------------------------------------------------------
 * The reference sizes its pair buffers from the pair total on the host (gstex.py:1045-1052, 1127: a device-to-host
 * read and a stream synchronisation every render).  Capacity mode sizes them from a capacity instead and keeps the
 * total on the device:
 *   gstex_scan_offsets_guarded: gstex_scan_offsets, and the thread that writes the total offsets[n] also writes
 *     *step_flag = (total > capacity) ? 1.0f : 0.0f (first != 0: the step's first render; otherwise the larger of
 *     the two) and, when host_count != NULL, the total into host_count -- memory the device can write and the host
 *     reads (pinned, mapped) once the stream has passed the scan: no copy, no synchronisation;
 *   gstex_bin_sort_capped: gstex_bin_sort_ordered with n_isect = the capacity (buffers, workspace); the kernels read
 *     the total from offsets[n], and a total above the capacity leaves every tile empty (nothing is written past the
 *     buffers);
 *   gstex_adam_step_guarded: gstex_adam_step_scaled that does nothing when *skip != 0 (an overflowed step's update
 *     is skipped on the device; the host grows the capacity when it sees the total).
 * The raster entry points take the capacity as n_isect (it only sizes the aux layout and the backward's grid, whose
 * surplus units exit at once). */
typedef struct gstex_pair_guard {
    int64_t capacity;
    float* step_flag;
    int32_t* host_count; /* nullable */
    int32_t first;
} gstex_pair_guard;
/* n device-writable host words (hipHostMalloc, mapped; zeroed): *host for the host, *device for
 * gstex_pair_guard.host_count.  Freed with gstex_host_words_free(host). */
int gstex_host_words_alloc(int32_t n, int32_t** host, int32_t** device);
int gstex_host_words_free(int32_t* host);

/* Lightweight events (ABI 14).  kind GSTEX_EVENT_TIMING: timing only, created with hipEventDisableSystemFence -- no
 * system-scope release / acquire (an L2 writeback and invalidate) when recorded, so a pair around a kernel measures it
 * without perturbing the loop it sits in (a default-event pair around each raster launch cost ~10 us of device time per
 * pair in bench.py's A/B); not for host synchronisation.  kind GSTEX_EVENT_ORDER: no timing, a device-scope release
 * (hipEventReleaseToDevice) -- for ordering one stream after another on the same device (gstex_stream_wait_event).
 * elapsed: milliseconds between two recorded, completed timing events. */
#define GSTEX_EVENT_TIMING 0
#define GSTEX_EVENT_ORDER 1
int gstex_event_create(int32_t kind, void** event);
int gstex_event_record(void* event, void* stream);
int gstex_event_elapsed(void* start, void* end, float* ms);
int gstex_stream_wait_event(void* stream, void* event);
int gstex_event_destroy(void* event);
int gstex_scan_offsets_guarded(int32_t n, const int32_t* num_tiles_hit, int32_t* offsets, void* workspace,
                               size_t workspace_bytes, const gstex_pair_guard* guard, void* stream);
int gstex_bin_sort_capped(int32_t n, int64_t capacity, const float* centers, const float* extents,
                          const float* depths, const int32_t* num_tiles_hit, const int32_t* offsets,
                          int32_t H, int32_t W, int32_t block, int32_t* tile_ranges, int32_t* sorted_ids,
                          int32_t* sorted_slots, int32_t* tile_order, void* workspace, size_t workspace_bytes,
                          void* stream);

/* Largest-first launch order of the tiles: tile_order[n_tiles] lists the tiles by descending
 * pair count (ties by tile index).  Pass it to gstex_raster_fwd / gstex_texture_edit, whose
 * workgroups the hardware dispatches in launch order round-robin over the 8 XCDs; NULL there
 * means row-major order.  Scheduling only: outputs do not depend on it.  Above 16384 tiles the
 * order is row-major. */
int gstex_tile_order(int32_t n_tiles, const int32_t* tile_ranges, int32_t* tile_order, void* stream);

/* ---- rasterizer --------------------------------------------------------------------- */
/* Builds the per-splat raster record table records[n][GSTEX_REC_FLOATS].
 * hp_records (ABI 18; nullable = none): a device double[n][GSTEX_HP_DOUBLES] buffer.  A splat whose normal is within
 * ~6 degrees of edge-on to its view direction (|n . d| < 0.1) is then marked near edge-on -- the sign bit of its
 * record opacity is set (every kernel reads the magnitude) -- and its row g receives the fp64 affine homography (A, B,
 * Pz), anchor and depth row; other rows are not written.  Pass the same buffer to gstex_raster_fwd(_zero) and
 * gstex_raster_bwd(_zero), which evaluate those splats' pairs from it (the offset from the anchor and the homogeneous
 * point in fp64, rounded once: their fp32 evaluation is ill-conditioned).  gstex_texture_edit ignores
 * the marks (pass records built without hp_records). */
int gstex_raster_setup(int32_t n, const float* means, const float* scales, float glob_scale,
                       const float* quats, const float* rgbs, const float* opacities,
                       const float* centers, const float* uv0, const float* umap,
                       const float* vmap, const int32_t* texture_dims,
                       const int32_t* num_tiles_hit, const gstex_camera* cam, float* records,
                       double* hp_records, void* stream);
/* Texel values: the texels are read as tex_scale * texture + tex_bias (1, 0 = as stored), so a caller
 * that keeps SH-DC coefficients (gstex.py:1119 passes SH2RGB(texture_dc) = 0.28209 x + 0.5) can pass the
 * store itself; the backward's v_texture is then the gradient w.r.t. the stored values. */
/* Forward composite. Outputs are [H][W][k] row-major. state[H*W][4] = {T_final, M1, M2,
 * last_contributor (as int bits)} is saved for the backward pass. background is a device
 * float[3] (or NULL = black) added as T_final * background.  out_depth, out_reg and out_normal may be
 * NULL together (geometric outputs not produced; the backward then takes no gradient for them).
 * aux (NULL = no backward follows): a gstex_raster_aux_bytes(n_isect, n_tiles, channels) device workspace the
 * forward fills for the backward -- its per-wave cull bits (per tile, 8x8 pixel quadrant and tile-list position),
 * per backward unit (tile, quadrant, segment of 256 list positions) the number of splats it evaluated, and
 * per-pixel checkpoints (transmittance and accumulators) at the segment boundaries of deep lists.  Pass the same
 * aux, untouched, to gstex_raster_bwd.
 * hp_records (ABI 18, nullable): gstex_raster_setup's near-edge-on rows -- the marked splats' pairs are then evaluated
 * from them (p in fp64, rounded once); pass the same buffer to the backward, which must take the same decisions.
 * NULL: every pair from the fp32 record (the marks ignored). */
int gstex_raster_fwd(const gstex_camera* cam, int32_t channels, int32_t settings,
                     const float* background, const float* records, const double* hp_records,
                     const int32_t* tile_ranges,
                     const int32_t* tile_order, const int32_t* sorted_ids, const float* texture,
                     int64_t n_texels, float tex_scale, float tex_bias,
                     float* out_img, float* out_depth, float* out_reg, float* out_alpha,
                     float* out_tex, float* out_normal, float* state, int64_t n_isect, void* aux,
                     void* stream);
/* The same, also zeroing zero_buf[0, zero_floats) and zero_buf2[0, zero_floats2) (ABI 11; NULL / 0 = none): the
 * buffers the backward accumulates into (the texel gradient, the fast mode's per-splat partials), cleared by the
 * forward's grid with streaming stores the raster work hides (no separate fills). */
int gstex_raster_fwd_zero(const gstex_camera* cam, int32_t channels, int32_t settings,
                          const float* background, const float* records, const double* hp_records,
                          const int32_t* tile_ranges,
                          const int32_t* tile_order, const int32_t* sorted_ids, const float* texture,
                          int64_t n_texels, float tex_scale, float tex_bias,
                          float* out_img, float* out_depth, float* out_reg, float* out_alpha,
                          float* out_tex, float* out_normal, float* state, int64_t n_isect, void* aux,
                          float* zero_buf, int64_t zero_floats, float* zero_buf2, int64_t zero_floats2,
                          void* stream);
size_t gstex_raster_aux_bytes(int64_t n_isect, int32_t n_tiles, int32_t channels);
/* Launch order of n_units backward units: unit_key = cost (bits 0-23, clamped to 1023) | XCD group (bits 24-26).
 * Units of cost 0 get no position; the others are sorted by descending cost within their group and the groups
 * interleaved (k-th unit of group g at position 8 k + g: round-robin dispatch puts it on XCD g), or, when the
 * groups are too uneven (8 x the largest group > n_units), sorted by descending cost overall.  unit_order[n_units]
 * holds -1 at unused positions; order within equal costs is unspecified.  scratch =
 * gstex_unit_order_scratch_words() int32 of device workspace.  gstex_raster_bwd calls it on its aux. */
int gstex_unit_order(int32_t n_units, const int32_t* unit_key, int32_t* unit_order, int32_t* scratch,
                     void* stream);
size_t gstex_unit_order_scratch_words(void);
/* Backward composite. Needs the forward state and the forward's aux (required; the backward also writes its
 * launch order into it).  Any of v_img ... v_normal may be NULL (that output's gradient is zero).  Texel blocks
 * that run past n_texels (corrupt texture_dims) are neither read nor written.  One wave per backward unit (tile,
 * 8x8 pixel quadrant q, segment): for every pair (emission slot s) the quadrant contributes to, writes the row
 * partials[(4 s + q) * R ...] (n_isect * 4 rows of R floats allocated; rows of pairs a quadrant does not reach are
 * never written) and sets byte q of row_flags[s] (n_isect uint32 words, zeroed by this call on the stream);
 * accumulates (+=) texel gradients into v_texture[n_texels][C].  R = GSTEX_PARTIAL_FLOATS_PHOTO (24) when neither
 * v_depth nor v_normal is given and v_reg is NULL or distortion (settings bit 10) is off -- the photometric training
 * step -- else GSTEX_PARTIAL_FLOATS (32); pass the same R to gstex_raster_setup_bwd(_aabb) as row_floats.
 * row_flags == NULL (ABI 9, the fast mode): instead of rows, every (pair, quadrant) sum is added with float
 * atomics into partials[g * R ...], an (n_splats, R) accumulator the caller has zeroed -- no per-pair rows, no
 * summing pass in setup_bwd; the splat gradients then depend on the atomics' order in their last bits (as the
 * texel gradients always do).  With row_flags the splat gradients are bitwise reproducible.
 * hp_records (ABI 18, nullable): the forward's hp_records (the same pairs evaluated the same way). */
int gstex_raster_bwd(const gstex_camera* cam, int32_t channels, int32_t settings,
                     const float* background, const float* records, const double* hp_records,
                     const int32_t* tile_ranges,
                     const int32_t* sorted_ids, const int32_t* sorted_slots, const float* texture,
                     int64_t n_texels, float tex_scale, float tex_bias, const float* state,
                     const float* v_img, const float* v_depth, const float* v_reg, const float* v_alpha,
                     const float* v_tex, const float* v_normal, int64_t n_isect, float* partials,
                     uint32_t* row_flags, float* v_texture, void* aux, void* stream);
/* gstex_raster_bwd that also zeroes zero_buf[0, zero_floats) with its grid (ABI 17): a persistent gradient buffer of
 * the NEXT step (gstex_amd.fused double-buffers the texel gradient: this backward accumulates into v_texture and zeroes
 * the other buffer, which the next step's backward accumulates into) -- instead of the forward's zeroing
 * (gstex_raster_fwd_zero).  zero_buf must not be v_texture. */
int gstex_raster_bwd_zero(const gstex_camera* cam, int32_t channels, int32_t settings, const float* background,
                          const float* records, const double* hp_records, const int32_t* tile_ranges,
                          const int32_t* sorted_ids,
                          const int32_t* sorted_slots, const float* texture, int64_t n_texels, float tex_scale,
                          float tex_bias, const float* state, const float* v_img, const float* v_depth,
                          const float* v_reg, const float* v_alpha, const float* v_tex, const float* v_normal,
                          int64_t n_isect, float* partials, uint32_t* row_flags, float* v_texture, void* aux,
                          float* zero_buf, int64_t zero_floats, void* stream);
/* Sums each splat's flagged partial rows (slot-major, quadrant-minor order: bitwise reproducible) and chains
 * them to the splat parameters. Outputs are overwritten.  partials is consumed: each splat's sums are written
 * over its first row (the rows are backward scratch, not read again).  row_flags == NULL: partials is the
 * backward's (n, row_floats) per-splat accumulator (gstex_raster_bwd without row_flags), chained directly.
 * n_rows (ABI 15): the pair capacity the rows were allocated for (n_rows * 4 rows), or -1 when offsets[n] is
 * known to fit; with capacity-sized pair buffers (gstex_bin_sort_capped) a total offsets[n] > n_rows means the
 * binning left every tile empty, and every splat is then chained as pair-free (zero gradients) without reading
 * rows past the allocation. */
int gstex_raster_setup_bwd(int32_t n, const float* means, const float* scales, float glob_scale,
                           const float* quats, const float* opacities, const float* umap,
                           const float* vmap, const int32_t* num_tiles_hit,
                           const int32_t* offsets, float* partials, const uint32_t* row_flags,
                           int32_t row_floats, int64_t n_rows, const gstex_camera* cam, float* v_means, float* v_scales,
                           float* v_quats, float* v_rgbs, float* v_opacities, float* v_centers,
                           float* v_uv0, void* stream);
/* gstex_raster_setup_bwd with gstex_aabb_2d_bwd folded in: for callers whose centres came from
 * gstex_aabb_2d on these same means / scales / quats (glob_scale, camera), the centre gradient is chained
 * through the AABB centre here and added to v_means / v_scales / v_quats (bit-identical to running
 * gstex_aabb_2d_bwd separately and adding the two results); v_centers is still written. */
int gstex_raster_setup_bwd_aabb(int32_t n, const float* means, const float* scales, float glob_scale,
                                const float* quats, const float* opacities, const float* umap,
                                const float* vmap, const int32_t* num_tiles_hit,
                                const int32_t* offsets, float* partials, const uint32_t* row_flags,
                                int32_t row_floats, int64_t n_rows, const gstex_camera* cam, float* v_means,
                                float* v_scales,
                                float* v_quats, float* v_rgbs, float* v_opacities, float* v_centers,
                                float* v_uv0, void* stream);

/* ---- spherical harmonics (degree <= 4) ------------------------------------------------- */
int gstex_sh_fwd(int32_t n, int32_t degree, int32_t n_coeffs, const float* viewdirs,
                 const float* coeffs, float* colors, void* stream);
int gstex_sh_bwd(int32_t n, int32_t degree, int32_t n_coeffs, const float* viewdirs,
                 const float* v_colors, float* v_coeffs, void* stream);

/* ---- jagged texture resample ------------------------------------------------------------ */
int gstex_texture_sample(int64_t n_query, int32_t channels, const int32_t* query_dims,
                         const float* texture, int64_t n_texels, const float* uv, float* out,
                         void* stream);
int gstex_texture_sample_bwd(int64_t n_query, int32_t channels, const int32_t* query_dims,
                             int64_t n_texels, const float* uv, const float* v_out,
                             float* v_texture, void* stream);

/* texture_edit (gstex.py:579-606, viewer paint tool): traverse each pixel's splats as
 * gstex_raster_fwd does (records from gstex_raster_setup, same tile lists/order); every counted pair
 * whose hit depth z satisfies depth_lo <= z <= depth_hi adds, to each of its 4 bilinear texels with
 * weight b and compositing weight w = alpha * T,  b * w * (a*r, a*g, a*b, a, 1)  to out[texel][5]
 * (ACCUMULATES: zero out first).  edit_rgb [H][W][3], edit_alpha/depth_lo/depth_hi [H][W]. */
int gstex_texture_edit(const gstex_camera* cam, int32_t settings, const float* records,
                       const int32_t* tile_ranges, const int32_t* tile_order, const int32_t* sorted_ids,
                       const float* edit_rgb, const float* edit_alpha, const float* depth_lo,
                       const float* depth_hi, int64_t n_texels, float* out, void* stream);

/* ---- splat activations (train-step support) ---------------------------- */
/* Per splat: quats_n = q/|q|; scales = (clamp(exp(s0),1e-9), clamp(exp(s1),1e-9), 1e-5*mean of those);
 * opacities = sigmoid(o); uv0 = 0.5, umap/vmap = mappings[:,0/1] * R(normalize(quats_n))[:, 0/1];
 * viewdirs = normalize(means - campos).  mappings is [n][mappings_stride] (>= 2); campos a device float[3];
 * quats / quats_n / v_quats 16-byte aligned.  The backward writes v_quats (raw quaternions), v_log_scales
 * (third axis 0: detached) and v_opac_logits; a NULL upstream gradient counts as zero and a NULL output
 * is skipped. */
int gstex_activate_fwd(int32_t n, const float* means, const float* quats, const float* log_scales,
                       const float* opac_logits, const float* mappings, int32_t mappings_stride,
                       const float* campos, float* quats_n, float* scales, float* opacities, float* uv0,
                       float* umap, float* vmap, float* viewdirs, void* stream);
int gstex_activate_bwd(int32_t n, const float* quats, const float* log_scales, const float* opacities,
                       const float* v_quats_n, const float* v_scales, const float* v_opacities,
                       float* v_quats, float* v_log_scales, float* v_opac_logits, void* stream);
/* SH colour from the non-DC coefficients only (the caller zeroes the DC term, gstex.py:1100):
 * coeffs_rest[n][n_rest][3] holds bases 1..n_rest; same result as gstex_sh_fwd on [0, coeffs_rest]. */
int gstex_sh_rest_fwd(int32_t n, int32_t degree, int32_t n_rest, const float* viewdirs,
                      const float* coeffs_rest, float* colors, void* stream);
int gstex_sh_rest_bwd(int32_t n, int32_t degree, int32_t n_rest, const float* viewdirs,
                      const float* v_colors, float* v_coeffs_rest, void* stream);

/* ---- photometric loss (train-step support) --------------------------------- */
/* rgb = clamp(img + tex[..., 0:3] + (1 - alpha) * background, 0, 1)      (gstex.py:1204-1205)
 * loss = (1 - ssim_lambda) * mean|gt - rgb| + ssim_lambda * (1 - SSIM(gt, rgb))  (gstex.py:1301-1322)
 * SSIM as pytorch_msssim: separable 11-tap window (window[11], host fp32), valid filtering,
 * C1 = 0.01^2, C2 = 0.03^2, mean over the (H-10) x (W-10) x 3 map.  Images are [H][W][k] row-major
 * device fp32; tex has C >= 3 channels (only 0..2 enter the loss).  loss_out (device float[3]) =
 * {loss, L1, SSIM}; rgb_out may be NULL.  The forward leaves in the workspace what the backward reads:
 * pass the same workspace to gstex_loss_bwd.  grad_loss is a device scalar (the loss's upstream
 * gradient); d_img, d_tex (channels >= 3 zero) and d_alpha are overwritten. */
size_t gstex_loss_workspace_size(int32_t H, int32_t W);
int gstex_loss_fwd(int32_t H, int32_t W, int32_t C, const float* img, const float* tex, const float* alpha,
                   const float* background, const float* gt, const float* window, float ssim_lambda,
                   float* rgb_out, float* loss_out, void* workspace, size_t workspace_bytes, void* stream);
int gstex_loss_bwd(int32_t H, int32_t W, int32_t C, const float* img, const float* tex, const float* alpha,
                   const float* background, const float* gt, const float* window, float ssim_lambda,
                   const float* grad_loss, float* d_img, float* d_tex, float* d_alpha, void* workspace,
                   size_t workspace_bytes, void* stream);

/* ---- optimizer (train-step support) ----------------------------------- */
/* One launch of torch.optim.Adam (no weight decay, no amsgrad) over up to GSTEX_ADAM_MAX_TENSORS
 * fp32 tensors.  Per tensor the host supplies step_size = lr / (1 - beta1^t) and
 * bias_correction2_sqrt = sqrt(1 - beta2^t) for that tensor's own step t.  Updates param,
 * exp_avg and exp_avg_sq in place. */
#define GSTEX_ADAM_MAX_TENSORS 16
typedef struct gstex_adam_tensor {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t numel;
    float step_size;
    float bias_correction2_sqrt;
} gstex_adam_tensor;
int gstex_adam_step(int32_t n_tensors, const gstex_adam_tensor* tensors, double beta1, double beta2,
                    double eps, void* stream);
/* gstex_adam_step with flags: GSTEX_ADAM_ZERO_GRAD also writes zeros over each gradient after reading it (so the
 * next backward can accumulate into the same buffer without a separate fill; the update may then run on a side
 * stream, overlapped with the next step's preprocessing).  Not in the reference (torch.optim.Adam + zero_grad). */
#define GSTEX_ADAM_ZERO_GRAD 1
/* flags bits 8..23: cap on the launch's workgroups (0 = one per 1024 elements), each looping over the chunks; a
 * capped grid (e.g. one workgroup per CU) still streams at near full HBM bandwidth while leaving most of every CU's
 * wave slots to kernels of another stream.  GSTEX_ADAM_GRID(n) builds the field. */
#define GSTEX_ADAM_GRID_SHIFT 8
#define GSTEX_ADAM_GRID(n) (((n) & 0xFFFF) << GSTEX_ADAM_GRID_SHIFT)
int gstex_adam_step_ex(int32_t n_tensors, const gstex_adam_tensor* tensors, double beta1, double beta2,
                       double eps, int32_t flags, void* stream);
/* gstex_adam_step_ex with every gradient read as grad * grad_scale, grad_scale in (0, 1] (ABI 7): a data-parallel
 * step passes 1 / world_size and skips the separate averaging pass over the all-reduced gradient buffer (the same
 * fp32 product, so the update is bit-identical).  Replaces, with GStex's GradSync, the 1 / world averaging of the
 * reference's DDP (pipelines/base_pipeline.py:281-283). */
int gstex_adam_step_scaled(int32_t n_tensors, const gstex_adam_tensor* tensors, double beta1, double beta2,
                           double eps, int32_t flags, float grad_scale, void* stream);
/* gstex_adam_step_scaled that reads *skip (a device float, nullable = never) first and updates nothing when it is
 * non-zero: the pair-capacity guard's step flag (gstex_scan_offsets_guarded), all-reduced with the gradients in
 * data-parallel training so that every rank skips the same steps.  ABI 13. */
int gstex_adam_step_guarded(int32_t n_tensors, const gstex_adam_tensor* tensors, double beta1, double beta2,
                            double eps, int32_t flags, float grad_scale, const float* skip, void* stream);

/* ---- training-step prologue (ABI 17; not in the reference) ------------------------------------------------------
 * One host call for the launches a photometric training render makes before its raster forward: the outputs of
 * gstex_activate_fwd, gstex_preprocess (the camera without c2w), gstex_sh_rest_fwd and gstex_scan_offsets_guarded --
 * bit-identical, computed by one per-splat kernel (the same device functions on the same values) and a one-launch
 * scan -- then gstex_raster_setup (glob_scale 1) and gstex_bin_sort_capped as called per op (gstex_amd.fused: the
 * trainer's render without ~0.2 ms of per-launch host overhead, which a step that starts on an idle device waits for,
 * and four launches fewer).  All pointers are device pointers; the buffers are sized as the per-op entry points
 * require (block = 16), scan_workspace as gstex_train_prologue_scan_bytes(n). */
typedef struct gstex_train_prologue_args {
    int32_t n;
    int32_t sh_degree;
    int32_t n_rest;
    int32_t map_cols;
    int64_t capacity;
    gstex_camera cam;
    gstex_pair_guard guard;
    const float* means;
    const float* quats;
    const float* log_scales;
    const float* opac_logits;
    const float* mappings;
    const float* campos;
    const float* features_rest;
    const int32_t* texture_dims;
    float* quats_n;
    float* scales;
    float* opacities;
    float* uv0;
    float* umap;
    float* vmap;
    float* viewdirs;
    float* depths;
    float* centers;
    float* extents;
    int32_t* num_tiles_hit;
    float* rgbs;
    int32_t* offsets;
    void* scan_workspace;
    size_t scan_workspace_bytes;
    float* records;
    int32_t* tile_ranges;
    int32_t* sorted_ids;
    int32_t* sorted_slots;
    int32_t* tile_order;
    void* bin_workspace;
    size_t bin_workspace_bytes;
    void* raster_aux;        /* nullable: the raster forward's aux buffer (gstex_raster_aux_bytes(capacity, n_tiles,
                                raster_channels)), whose accumulated span the prologue zeroes -- pass
                                GSTEX_SETTING_AUX_ZEROED to the forward that follows */
    size_t raster_aux_bytes;
    int32_t raster_channels;
    double* hp_records;      /* nullable (ABI 18): gstex_raster_setup's near-edge-on fp64 rows, double[n][12] */
} gstex_train_prologue_args;
int gstex_train_prologue(const gstex_train_prologue_args* args, void* stream);
/* Bytes of scan_workspace gstex_train_prologue needs for n splats (>= gstex_scan_workspace_size(n): the fused
 * preprocessing kernel leaves one tile-count sum per 128 splats there for the one-launch offsets scan). */
size_t gstex_train_prologue_scan_bytes(int32_t n);

/* The photometric training render's backward after gstex_raster_bwd (fast mode: partials = the zeroed (n, 24)
 * per-splat accumulator rows it added into), in one call (ABI 17; gstex_amd.fused): gstex_raster_setup_bwd_aabb
 * (glob_scale 1, the camera with c2w), then gstex_activate_bwd and gstex_sh_rest_bwd on its outputs -- one kernel, the
 * same device functions on the same values (bit-identical), when the SH rows fit its LDS staging.  v_* are the
 * parameter gradients (written, not accumulated); v_*_act and v_centers / v_uv0 are scratch of n rows each (the
 * activated parameters' gradients, as the per-op calls write them). */
typedef struct gstex_train_epilogue_args {
    int32_t n;
    int32_t sh_degree;
    int32_t n_rest;
    gstex_camera cam;
    const float* means;
    const float* scales;     /* activated (gstex_activate_fwd) */
    const float* quats_n;    /* normalised */
    const float* quats;      /* raw parameter */
    const float* log_scales;
    const float* opacities;  /* activated */
    const float* umap;
    const float* vmap;
    const float* viewdirs;
    const int32_t* num_tiles_hit;
    const int32_t* offsets;
    float* partials;
    float* v_means;
    float* v_quats;
    float* v_log_scales;
    float* v_opac_logits;
    float* v_features_rest;
    float* v_scales_act;
    float* v_quats_n;
    float* v_rgbs;
    float* v_opacities_act;
    float* v_centers;
    float* v_uv0;
} gstex_train_epilogue_args;
int gstex_train_epilogue(const gstex_train_epilogue_args* args, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GSTEX_HIP_H */
