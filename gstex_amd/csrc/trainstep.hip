// trainstep.hip — the launches a photometric training render makes before its raster forward, as one host call
// (gstex_train_prologue, ABI 17; gstex_amd.fused).
//
// Per-op sequence (gstex_amd's per-op path): activate_fwd, preprocess, sh_rest_fwd (one thread per splat each), the
// guarded offsets scan (three launches: block sums, scan of the sums, final), raster_setup, bin_sort_capped.  Here:
//   train_splat_kernel  one thread per splat runs activate_splat -> preprocess_splat -> sh_colour -> splat_record
//                       (splat_math.h, the functions the per-op kernels call, on the same fp32 values: bit-identical
//                       outputs) and writes every per-op output incl. the raster record, plus the tile-count sum of
//                       its kSplatBlock (256)-splat block;
//   train_scan_kernel   the offsets scan in one launch: each 1024-splat scan tile starts from the sum of the block
//                       sums before it (kBlocksPerTile = 4 per tile; at most n / 256 L2-resident words), then scans its tile as
//                       binning.hip's scan_final_kernel does (same integers, same guard);
//                       its grid also zeroes the binning's tile counters and the raster forward's accumulated aux span
//                       (args.raster_aux), so neither needs its fill launch (GSTEX_SETTING_AUX_ZEROED);
// then the capped binning.  Seven launches fewer and no host time between the launches (the device waits through that
// whenever a step starts on an idle device, after a synchronisation).
#include "gstex_common.h"
#include "gstex_error.h"
#include "gstex_internal.h"
#include "splat_math.h"

using namespace gstex;

namespace {

// splats per workgroup of train_splat_kernel, whose SH coefficient rows are staged in LDS (cfg3: 30.8 us at 256, 33.9
// at 64, 34.9 at 128; unstaged rows 38.8-40.8 -- EXPERIMENTS.md)
constexpr int kSplatBlock = 256;
constexpr int kScanBlock = 256;
constexpr int kScanItems = 4;
constexpr int kScanTile = kScanBlock * kScanItems;  // = binning.hip's scan tile
constexpr int kBlocksPerTile = kScanTile / kSplatBlock;
// SH rows staged per workgroup within 64 KiB of LDS (256 splats: up to 21 rest coefficients, degree 3's 15; degree 4
// takes the per-op path)
constexpr int kMaxRest = 65536 / (kSplatBlock * 3 * 4);

__global__ __launch_bounds__(kSplatBlock) void train_splat_kernel(
    int n, int degree, int n_rest, const float* __restrict__ means, const float* __restrict__ quats,
    const float* __restrict__ log_scales, const float* __restrict__ opac_logits, const float* __restrict__ mappings,
    int map_stride, const float* __restrict__ campos, const float* __restrict__ coeffs_rest, CamArgs cam_args,
    int tiles_x, int tiles_y, int block, float* __restrict__ quats_n, float* __restrict__ scales,
    float* __restrict__ opacities, float* __restrict__ uv0, float* __restrict__ umap, float* __restrict__ vmap,
    float* __restrict__ viewdirs, float* __restrict__ depths, float* __restrict__ centers,
    float* __restrict__ extents, int32_t* __restrict__ nth, float* __restrict__ rgbs,
    const int32_t* __restrict__ tdims, float* __restrict__ records, double* __restrict__ hp_records,
    int32_t* __restrict__ block_sums) {
    extern __shared__ float s_c[];
    __shared__ int s_wave[kSplatBlock / 64];
    const Camera cam = load_camera(cam_args);
    const int t = threadIdx.x;
    const int i0 = blockIdx.x * kSplatBlock;
    const int cnt = min(kSplatBlock, n - i0);
    const int kw = n_rest * 3;
    sh_copy_span<kSplatBlock>(s_c, coeffs_rest + (size_t)i0 * kw, cnt * kw);
    __syncthreads();
    int count = 0;
    if (t < cnt) {
        const int i = i0 + t;
        const float mx = means[3 * i], my = means[3 * i + 1], mz = means[3 * i + 2];
        const Activated a = activate_splat(reinterpret_cast<const float4*>(quats)[i], log_scales[3 * i],
                                           log_scales[3 * i + 1], opac_logits[i], mappings[(size_t)map_stride * i],
                                           mappings[(size_t)map_stride * i + 1], mx, my, mz, campos);
        store_activated(i, a, quats_n, scales, opacities, uv0, umap, vmap, viewdirs);
        const Preprocessed p = preprocess_splat(cam, mk3(mx, my, mz), a.s0, a.s1, 1.0f, a.q, tiles_x, tiles_y, block);
        depths[i] = p.depth;
        centers[2 * i] = p.cx;
        centers[2 * i + 1] = p.cy;
        extents[2 * i] = p.ex;
        extents[2 * i + 1] = p.ey;
        nth[i] = p.nth;
        count = p.nth;
        float r0, r1, r2;
        sh_colour(degree, 1, a.vd[0], a.vd[1], a.vd[2], s_c + t * kw - 3, r0, r1, r2);
        rgbs[3 * i] = r0;
        rgbs[3 * i + 1] = r1;
        rgbs[3 * i + 2] = r2;
        if (p.nth > 0) {  // the raster record of a splat that hits a tile (as setup_kernel)
            const float rgb[3] = {r0, r1, r2};
            const float uv[2] = {0.5f, 0.5f};
            const int32_t td[3] = {tdims[3 * i], tdims[3 * i + 1], tdims[3 * i + 2]};
            splat_record(cam, mx, my, mz, a.s0, a.s1, 1.0f, a.q, rgb, a.opacity, p.cx, p.cy, uv, a.um, a.vm, td,
                         records + (size_t)i * GSTEX_REC_FLOATS, hp_records ? hp_records + (size_t)i * H_FIELDS : nullptr);
        }
    }
    int total;
    block_excl_scan<kSplatBlock>(count, s_wave, &total);
    if (t == 0) block_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanBlock) void train_scan_kernel(int n, const int32_t* __restrict__ in,
                                                                const int32_t* __restrict__ block_sums,
                                                                int32_t* __restrict__ out, const ScanGuard guard,
                                                                uint4* __restrict__ z0, int z0n,
                                                                uint4* __restrict__ z1, int z1n) {
    __shared__ int s_wave[kScanBlock / 64];
    // side job: the binning's tile counters and the raster forward's accumulated aux span (their fill launches)
    for (int k = blockIdx.x * kScanBlock + threadIdx.x; k < z0n + z1n; k += gridDim.x * kScanBlock) {
        if (k < z0n) z0[k] = make_uint4(0u, 0u, 0u, 0u);
        else z1[k - z0n] = make_uint4(0u, 0u, 0u, 0u);
    }
    const int tile = blockIdx.x;
    int pre = 0;
    for (int j = threadIdx.x; j < tile * kBlocksPerTile; j += kScanBlock) pre += block_sums[j];
    int prefix;
    block_excl_scan<kScanBlock>(pre, s_wave, &prefix);
    const int base = tile * kScanTile + threadIdx.x * kScanItems;
    int vals[kScanItems];
    int v = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        vals[k] = (base + k < n) ? in[base + k] : 0;
        v += vals[k];
    }
    int total;
    int ex = block_excl_scan<kScanBlock>(v, s_wave, &total) + prefix;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        if (base + k < n) out[base + k] = ex;
        ex += vals[k];
    }
    if (tile == gridDim.x - 1 && threadIdx.x == kScanBlock - 1) {
        out[n] = ex;
        apply_guard(guard, ex);
    }
}

size_t block_sums_bytes(int n) { return (size_t)div_up(n, kSplatBlock) * sizeof(int32_t); }

}  // namespace

extern "C" size_t gstex_train_prologue_scan_bytes(int32_t n) {
    const size_t per_op = gstex_scan_workspace_size(n);
    const size_t fused = block_sums_bytes(n < 0 ? 0 : n);
    return per_op > fused ? per_op : fused;
}

extern "C" int gstex_train_prologue(const gstex_train_prologue_args* a, void* stream) {
    GSTEX_REQUIRE(a, "gstex_train_prologue: null arguments");
    GSTEX_REQUIRE(a->n >= 0 && a->capacity >= 0, "gstex_train_prologue: invalid sizes (n %d)", a->n);
    GSTEX_REQUIRE(a->scan_workspace && a->scan_workspace_bytes >= gstex_train_prologue_scan_bytes(a->n),
                  "gstex_train_prologue: scan workspace too small (%zu < %zu bytes)", a->scan_workspace_bytes,
                  gstex_train_prologue_scan_bytes(a->n));
    gstex_camera pre = a->cam;  // preprocessing takes the view without c2w (as gstex_amd.ops.preprocess)
    pre.c2w = nullptr;
    GSTEX_REQUIRE(pre.block > 0 && pre.H > 0 && pre.W > 0, "gstex_train_prologue: invalid camera");
    {  // the spans zeroed below lie inside the buffers the caller sized
        const int n_tiles = ((pre.W + pre.block - 1) / pre.block) * ((pre.H + pre.block - 1) / pre.block);
        GSTEX_REQUIRE(a->bin_workspace &&
                          a->bin_workspace_bytes >= gstex_bin_workspace_size(a->n, a->capacity, n_tiles),
                      "gstex_train_prologue: bin workspace too small");
        GSTEX_REQUIRE(!a->raster_aux || (a->raster_channels >= 1 && a->raster_channels <= 8 &&
                                         a->raster_aux_bytes >= gstex_raster_aux_bytes(a->capacity, n_tiles,
                                                                                       a->raster_channels)),
                      "gstex_train_prologue: raster aux buffer too small or channels out of range");
    }
    int rc;
    const bool fused = a->n > 0 && a->sh_degree >= 1 && a->sh_degree <= 4 && a->n_rest <= kMaxRest &&
                       a->n_rest >= (a->sh_degree + 1) * (a->sh_degree + 1) - 1 && a->map_cols >= 2;
    if (fused) {
        GSTEX_REQUIRE(a->means && a->quats && a->log_scales && a->opac_logits && a->mappings && a->campos &&
                          a->features_rest && a->quats_n && a->scales && a->opacities && a->uv0 && a->umap &&
                          a->vmap && a->viewdirs && a->depths && a->centers && a->extents && a->num_tiles_hit &&
                          a->rgbs && a->offsets && a->texture_dims && a->records && a->cam.viewmat,
                      "gstex_train_prologue: null pointer");
        GSTEX_REQUIRE(((reinterpret_cast<uintptr_t>(a->quats) | reinterpret_cast<uintptr_t>(a->quats_n)) & 15) == 0,
                      "gstex_train_prologue: quaternions must be 16-byte aligned");
        hipStream_t st = as_stream(stream);
        const int tx = (pre.W + pre.block - 1) / pre.block, ty = (pre.H + pre.block - 1) / pre.block;
        int32_t* sums = static_cast<int32_t*>(a->scan_workspace);
        train_splat_kernel<<<div_up(a->n, kSplatBlock), kSplatBlock,
                             (size_t)kSplatBlock * a->n_rest * 3 * sizeof(float), st>>>(
            a->n, a->sh_degree, a->n_rest, a->means, a->quats, a->log_scales, a->opac_logits, a->mappings,
            a->map_cols, a->campos, a->features_rest, to_device_camera(a->cam), tx, ty, pre.block, a->quats_n,
            a->scales, a->opacities, a->uv0, a->umap, a->vmap, a->viewdirs, a->depths, a->centers, a->extents,
            a->num_tiles_hit, a->rgbs, a->texture_dims, a->records, a->hp_records, sums);
        const ScanGuard g{(long long)a->guard.capacity, a->guard.step_flag, a->guard.host_count,
                          a->guard.first ? 1 : 0};
        const ZeroSpan zb = bin_count_span(a->bin_workspace, tx * ty, a->capacity);
        const ZeroSpan za = a->raster_aux ? raster_aux_zero_span(a->raster_aux, a->capacity, tx * ty,
                                                                 a->raster_channels)
                                          : ZeroSpan{nullptr, 0};
        GSTEX_REQUIRE(((reinterpret_cast<uintptr_t>(zb.ptr) | reinterpret_cast<uintptr_t>(za.ptr) | zb.bytes | za.bytes) &
                       15) == 0, "gstex_train_prologue: workspaces must be 16-byte aligned");
        train_scan_kernel<<<div_up(a->n, kScanTile), kScanBlock, 0, st>>>(
            a->n, a->num_tiles_hit, sums, a->offsets, g, static_cast<uint4*>(zb.ptr), (int)(zb.bytes / 16),
            static_cast<uint4*>(za.ptr), (int)(za.bytes / 16));
        rc = launch_status("gstex_train_prologue");
    } else {  // the per-op entry points (n = 0, or an SH layout the fused kernel does not stage)
        rc = gstex_activate_fwd(a->n, a->means, a->quats, a->log_scales, a->opac_logits, a->mappings, a->map_cols,
                                a->campos, a->quats_n, a->scales, a->opacities, a->uv0, a->umap, a->vmap,
                                a->viewdirs, stream);
        if (rc) return rc;
        rc = gstex_preprocess(a->n, a->means, a->scales, 1.0f, a->quats_n, &pre, a->depths, a->centers, a->extents,
                              a->num_tiles_hit, stream);
        if (rc) return rc;
        rc = gstex_sh_rest_fwd(a->n, a->sh_degree, a->n_rest, a->viewdirs, a->features_rest, a->rgbs, stream);
        if (rc) return rc;
        rc = gstex_scan_offsets_guarded(a->n, a->num_tiles_hit, a->offsets, a->scan_workspace,
                                        a->scan_workspace_bytes, &a->guard, stream);
        if (rc == 0 && a->raster_aux) {  // (the caller passes GSTEX_SETTING_AUX_ZEROED to the forward)
            const int tx = (pre.W + pre.block - 1) / pre.block, ty = (pre.H + pre.block - 1) / pre.block;
            const ZeroSpan za = raster_aux_zero_span(a->raster_aux, a->capacity, tx * ty, a->raster_channels);
            if (hipMemsetAsync(za.ptr, 0, za.bytes, as_stream(stream)) != hipSuccess)
                return launch_status("gstex_train_prologue (aux)");
        }
    }
    if (rc) return rc;
    if (!fused) {  // (the fused kernel wrote the records)
        rc = gstex_raster_setup(a->n, a->means, a->scales, 1.0f, a->quats_n, a->rgbs, a->opacities, a->centers, a->uv0,
                                a->umap, a->vmap, a->texture_dims, a->num_tiles_hit, &a->cam, a->records,
                                a->hp_records, stream);
        if (rc) return rc;
    }
    if (fused)  // the tile counters were zeroed by train_scan_kernel
        return bin_sort_capped_prezeroed(a->n, a->capacity, a->centers, a->extents, a->depths, a->offsets, a->cam.H,
                                         a->cam.W, a->cam.block, a->tile_ranges, a->sorted_ids, a->sorted_slots,
                                         a->tile_order, a->bin_workspace, a->bin_workspace_bytes, stream);
    return gstex_bin_sort_capped(a->n, a->capacity, a->centers, a->extents, a->depths, a->num_tiles_hit, a->offsets,
                                 a->cam.H, a->cam.W, a->cam.block, a->tile_ranges, a->sorted_ids, a->sorted_slots,
                                 a->tile_order, a->bin_workspace, a->bin_workspace_bytes, stream);
}
