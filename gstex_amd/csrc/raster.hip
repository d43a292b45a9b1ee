// raster.hip — forward / backward alpha-composite of per-primitive-textured 2D Gaussian splats.
//
// Replaces gstex_cuda.texture.texture_gaussians (forward at nerfstudio/models/gstex.py:1133-1162,
// backward through autograd at engine/trainer.py:460).  Semantics: SURVEY.md Appendix A and the
// comments of gstex_common.h; the CPU restatement is oracle/raster.py.
//
// MI355X layout:
//   * forward: one 256-thread workgroup (4 wave64, one 8x8 quadrant each) per 16x16 tile, launched in
//     descending pair-count order (gstex_tile_order); splat records are 128-B lines staged per batch in LDS as
//     [plane][splat] float4; each wave ballots the batch against its quadrant (exact ellipse-vs-rectangle
//     test), walks the set bits, early-outs per lane and per workgroup; it records for the backward (aux):
//     its cull bits, per-unit evaluation counts and per-pixel checkpoints at 256-position segment boundaries;
//   * backward: one wave64 workgroup per unit = (tile, 8x8 quadrant, segment), launched costliest first, no
//     barriers and no shared state between waves; a unit starts from the forward's checkpoint after its
//     segment and walks back to front; per visit the 24 splat partials are reduced across the wave with a
//     reduce-scatter butterfly (permlane32/16 swaps + DPP) and added into the splat's accumulator row with one
//     coalesced float-atomic instruction (deterministic mode: stored as the (pair, quadrant) row at the pair's
//     emission slot and summed in fixed order by setup_bwd); texel gradients go through a DPP segmented scan,
//     int32 fixed-point LDS staging of the splat's block and a flush of its non-zero entries with global fp32
//     atomics.
#include "gstex_common.h"
#include "gstex_error.h"
#include "gstex_internal.h"
#include "splat_math.h"  // splat_record
#include "raster_diag.h"  // diagnostic builds only (GSTEX_STATS counters); empty by default

using namespace gstex;

namespace {

constexpr int kThreads = kTilePixels;  // 256
#ifndef GSTEX_FWD_BATCH
#define GSTEX_FWD_BATCH 128
#endif
#ifndef GSTEX_SEG_W
// texel-gradient segment width in lanes: half a pixel row of the 8x8 quadrant (2 scan steps, twice the run tails of
// a whole row: measured 4% faster backward than 8, 2 is slower again)
#define GSTEX_SEG_W 4
#endif
#ifndef GSTEX_FAST_RCP
#define GSTEX_FAST_RCP 1  // v_rcp_f32 for backward divisions that feed no threshold decision
#endif
#ifndef GSTEX_FAST_EVAL
#define GSTEX_FAST_EVAL 1  // hardware v_exp_f32 / v_rcp_f32 in the pair evaluation (0: expf sequence, IEEE division)
#endif

#ifndef GSTEX_UNIT_COARSE
#define GSTEX_UNIT_COARSE 3  // backward unit-order cost buckets of 2^k visits (inside a bucket: about slot order,
                             // better L2 reuse of texel blocks). Measured: 3 same time, bwd fetch -18 %; 5, 6 slower
#endif
#ifndef GSTEX_FWD_OCC
#define GSTEX_FWD_OCC 6  // forward waves per SIMD the register allocation targets (measured: 8 at 64 VGPRs is slower; 5 with
                         // a record prefetch or a second pending texel set, both measured slower in round 5)
#endif
#ifndef GSTEX_XCD_MB
#define GSTEX_XCD_MB 2  // backward units of one 2x2-tile macro-block dispatched to one XCD (unit_order groups)
#endif
// Backward occupancy: waves per SIMD the register allocation targets, per instantiation.  The photometric
// training variant (C = 3, no geometry gradients) fits 7 (72 VGPRs, no spills; 8 forces 64 VGPRs with scratch
// spills and is 3 % slower); the others 5.  Measured: warming the next visit's record line with a scalar load
// during the current visit gains nothing (records hit in cache).
#ifndef GSTEX_BWD_WAVES_TRAIN
#define GSTEX_BWD_WAVES_TRAIN 7
#endif
#ifndef GSTEX_BWD_WAVES
#define GSTEX_BWD_WAVES 5
#endif
template <int C, bool GEO>
struct BwdShape {
    static constexpr bool kTrain = (C == 3 && !GEO);
    static constexpr int kWaves = kTrain ? GSTEX_BWD_WAVES_TRAIN : GSTEX_BWD_WAVES;
};
// Backward per-wave texel staging: one splat's texel block (h * w * C int32 fixed-point entries) at a time, 4 KiB
// per wave (341 texels at C = 3; cfg3's largest block is 169); a larger block adds its run tails straight to global
// memory.  Measured: 6 KiB staging 3 % slower than 4, 3 and 2 KiB (equal); int64 staging +0.15 ms.)
#ifndef GSTEX_TEX_STAGE
#define GSTEX_TEX_STAGE 1024
#endif
constexpr int kTexStage = GSTEX_TEX_STAGE;
constexpr int kFwdBatch = GSTEX_FWD_BATCH;
#ifndef GSTEX_FWD_DEFER
#define GSTEX_FWD_DEFER 1
#endif
constexpr bool kFwdDefer = GSTEX_FWD_DEFER;  // forward: texel gathers folded in one visit later (C = 3)
constexpr int kRecF4 = GSTEX_REC_FLOATS / 4;  // 8 float4 per record
#ifndef GSTEX_WORD_WAIT
#define GSTEX_WORD_WAIT 1  // backward: the visit loop's id wait hoisted to the word start (see raster_bwd_kernel)
#endif

// ------------------------------------------------------------------------------------------
// setup: per-splat record
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void setup_kernel(int n, const float* __restrict__ means,
                                                    const float* __restrict__ scales, float glob,
                                                    const float* __restrict__ quats,
                                                    const float* __restrict__ rgbs,
                                                    const float* __restrict__ opacities,
                                                    const float* __restrict__ centers,
                                                    const float* __restrict__ uv0,
                                                    const float* __restrict__ umap,
                                                    const float* __restrict__ vmap,
                                                    const int32_t* __restrict__ tdims,
                                                    const int32_t* __restrict__ nth, CamArgs cam_args,
                                                    float* __restrict__ rec_out, double* __restrict__ hp_out) {
    const Camera cam = load_camera(cam_args);
    int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= n) return;
    if (nth[g] <= 0) return;
    // the record, in fp64 (splat_math.h: the function the training prologue's fused kernel also calls)
    splat_record(cam, means[3 * g], means[3 * g + 1], means[3 * g + 2], scales[3 * g], scales[3 * g + 1], glob,
                 quats + 4 * g, rgbs + 3 * g, opacities[g], centers[2 * g], centers[2 * g + 1], uv0 + 2 * g,
                 umap + 3 * g, vmap + 3 * g, tdims + 3 * g, rec_out + (size_t)g * GSTEX_REC_FLOATS,
                 hp_out ? hp_out + (size_t)g * H_FIELDS : nullptr);
}

// ------------------------------------------------------------------------------------------
// shared per-(pixel, splat) evaluation
// ------------------------------------------------------------------------------------------
struct Rec {
    f3 A, B, Tw;
    float Pz;
    float x, y, opac, mark;  // opac = |R_OPAC|; mark = the raw word (sign bit: near edge-on, gstex_common.h kHpCos)
    float rgb[3], nrm[3];
    float tu0, auu, auv, tv0, avu, avv;
    int h, w, off;
    float xa, ya;
    float hm1, wm1;  // (float)(h - 1), (float)(w - 1)
};

// Record fields from its 8 float4 planes (gstex_common.h RecField)
__device__ __forceinline__ Rec rec_from_planes(float4 a, float4 b, float4 c, float4 d, float4 e, float4 f, float4 g,
                                               float4 q) {
    const float v[GSTEX_REC_FLOATS] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w,
                                       e.x, e.y, e.z, e.w, f.x, f.y, f.z, f.w, g.x, g.y, g.z, g.w, q.x, q.y, q.z, q.w};
    Rec r;
    r.A = f3{v[R_A], v[R_A + 1], v[R_A + 2]};
    r.B = f3{v[R_B], v[R_B + 1], v[R_B + 2]};
    r.Pz = v[R_PZ];
    r.Tw = f3{v[R_TW], v[R_TW + 1], v[R_TW + 2]};
    r.x = v[R_XY]; r.y = v[R_XY + 1];
    r.opac = fabsf(v[R_OPAC]);
    r.mark = v[R_OPAC];
    r.rgb[0] = v[R_RGB]; r.rgb[1] = v[R_RGB + 1]; r.rgb[2] = v[R_RGB + 2];
    r.tu0 = v[R_TU0]; r.auu = v[R_AUU]; r.auv = v[R_AUV]; r.tv0 = v[R_TV0]; r.avu = v[R_AVU]; r.avv = v[R_AVV];
    r.h = __float_as_int(v[R_H]); r.w = __float_as_int(v[R_W]); r.off = __float_as_int(v[R_OFF]);
    r.xa = v[R_XA]; r.ya = v[R_YA];
    r.nrm[0] = v[R_NRM]; r.nrm[1] = v[R_NRM + 1]; r.nrm[2] = v[R_NRM + 2];
    r.hm1 = v[R_HM1]; r.wm1 = v[R_WM1];
    return r;
}

// Pixel of thread tid inside a 16x16 tile and the wave's block of pixel centres.
struct WaveBlock { int px, py; float wx0, wx1, wy0, wy1; };  // w*: the cull box (pixel centres +- 0.05)
__device__ __forceinline__ WaveBlock wave_block(int tx, int ty, int tid) {
    WaveBlock b;
    const int w = tid >> 6, l = tid & 63;
    b.px = tx * kTile + (w & 1) * 8 + (l & 7);  // wave w covers the 8x8 quadrant (w & 1, w >> 1)
    b.py = ty * kTile + (w >> 1) * 8 + (l >> 3);
    // the cull box is wave-uniform: held in SGPRs (as VGPRs its four bounds were the allocator's first spill
    // candidates, reloaded from scratch by every record's cull test)
    auto uni = [](float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); };
    const float x0 = (float)(tx * kTile + (w & 1) * 8) + 0.5f, y0 = (float)(ty * kTile + (w >> 1) * 8) + 0.5f;
    b.wx0 = uni(x0 - 0.05f);
    b.wy0 = uni(y0 - 0.05f);
    b.wx1 = uni((x0 + 7.0f) + 0.05f);
    b.wy1 = uni((y0 + 7.0f) + 0.05f);
    return b;
}

__host__ __device__ __forceinline__ int fwd_grid(int tiles_x, int tiles_y) { return tiles_x * tiles_y; }

// Record j of a batch staged in LDS as [plane][splat] float4
template <int NB>
__device__ __forceinline__ Rec read_rec(const float4* s, int j) {
    return rec_from_planes(s[0 * NB + j], s[1 * NB + j], s[2 * NB + j], s[3 * NB + j], s[4 * NB + j], s[5 * NB + j],
                           s[6 * NB + j], s[7 * NB + j]);
}

// Visit-mask layout: tile t owns 64-bit words [ceil(start_t / 64) + t, + ceil(len_t / 64)) (disjoint across tiles);
// word i holds, for each of the 4 waves (interleaved: word * 4 + wave), one bit per tile-list position
// 64 i .. 64 i + 63: the forward's per-wave cull (the splat's contribution region meets the wave's block).
__host__ __device__ __forceinline__ size_t visit_mask_base(int start, int tile) {
    return (size_t)((start + 63) / 64) + (size_t)tile;
}

// Backward units: the backward splits each (tile, 8x8 quadrant) list at every kSegLen positions into segments, one
// wave each, so no wave walks more than kSegLen positions (a deep unit as one wave was the kernel's critical path).
// Segment k of tile t has slot seg_base(start_t, t) + k (disjoint across tiles, like the visit-mask words); unit =
// 4 slot + quadrant.  The forward records, per unit, the number of splats it evaluated (the backward's cost
// estimate and launch order), the tile of every slot, and per-pixel checkpoints: for each segment boundary it
// crosses with a lane still running, the state after the segment (T and the colour / texture / depth / normal /
// distortion accumulators), and for a wave whose last contributor lies past the first segment, its final
// accumulators in the slot of that last segment.  The backward of segment k starts from checkpoint k instead of
// the final state: T = T_k, and R = (back half of sum_j w_j g_j + T_final bg-term) / T_k from the accumulators.
#ifndef GSTEX_SEG_LEN
#define GSTEX_SEG_LEN 256
#endif
constexpr int kSegLen = GSTEX_SEG_LEN;
static_assert(kSegLen % 128 == 0, "segments end at forward batch boundaries");
__host__ __device__ __forceinline__ int seg_base(int start, int tile) { return (start + kSegLen - 1) / kSegLen + tile; }
__host__ __device__ __forceinline__ int ck_fields(int C) { return 4 + C + 6; }  // T, img[3], tex[C], D, nrm[3], M1, M2

struct AuxPtrs {
    unsigned long long* masks;
    int32_t* cost;       // [n_units] evaluation count | XCD group (2x2-tile macro-block) << 24
    int32_t* order;      // [n_units] (written by the backward)
    int32_t* order_ws;   // gstex_unit_order scratch
    int32_t* slot_tile;  // [n_slots]
    float* ckpt;         // [n_units][F][64]
    int F;
};
struct AuxLayout { size_t masks, cost, order, order_ws, slot_tile, ckpt, bytes; int64_t n_slots, n_units; int F; };
struct ZeroBufs { float* p[2]; int64_t n[2]; };  // buffers the forward's grid zeroes (gstex_raster_fwd_zero)
// The accumulation buffers a raster kernel's whole grid zeroes as a side job (gstex_raster_fwd_zero: the texel gradient
// and the splat-gradient sums of the backward that follows; gstex_raster_bwd_zero: the next step's texel gradient):
// plain streaming stores the VALU-bound raster kernels hide, instead of fill passes (or an Adam update's zero stores)
__device__ __forceinline__ void zero_bufs(const ZeroBufs& zb) {
    const int64_t nthr = (int64_t)gridDim.x * blockDim.x, t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        float* zp = zb.p[b];
        const int64_t zn = zb.n[b];
        if (!zp) continue;
        if ((reinterpret_cast<uintptr_t>(zp) & 15) == 0) {
            typedef float z4v __attribute__((ext_vector_type(4)));
            z4v* z4 = reinterpret_cast<z4v*>(zp);
            const z4v zero = {0.f, 0.f, 0.f, 0.f};
            for (int64_t i = t0; i < zn / 4; i += nthr) __builtin_nontemporal_store(zero, z4 + i);
            if (t0 < zn % 4) zp[zn / 4 * 4 + t0] = 0.0f;
        } else {
            for (int64_t i = t0; i < zn; i += nthr) zp[i] = 0.0f;
        }
    }
}
__host__ inline AuxLayout aux_layout(int64_t n_isect, int n_tiles, int C) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    AuxLayout a;
    a.n_slots = (n_isect + kSegLen - 1) / kSegLen + n_tiles + 1;
    a.n_units = a.n_slots * 4;
    a.F = ck_fields(C);
    size_t o = 0;
    a.masks = o; o = al(o + (((size_t)n_isect + 63) / 64 + (size_t)n_tiles + 1) * 4 * sizeof(uint64_t));
    a.cost = o; o = al(o + (size_t)a.n_units * 4);
    a.order = o; o = al(o + (size_t)a.n_units * 4);
    a.order_ws = o; o = al(o + gstex_unit_order_scratch_words() * 4);
    a.slot_tile = o; o = al(o + (size_t)a.n_slots * 4);
    a.ckpt = o; o = al(o + (size_t)a.n_units * a.F * 64 * sizeof(float));
    a.bytes = o;
    return a;
}
__host__ inline AuxPtrs aux_ptrs(void* aux, const AuxLayout& a) {
    char* b = (char*)aux;
    AuxPtrs p;
    p.masks = aux ? (unsigned long long*)(b + a.masks) : nullptr;
    p.cost = aux ? (int32_t*)(b + a.cost) : nullptr;
    p.order = aux ? (int32_t*)(b + a.order) : nullptr;
    p.order_ws = aux ? (int32_t*)(b + a.order_ws) : nullptr;
    p.slot_tile = aux ? (int32_t*)(b + a.slot_tile) : nullptr;
    p.ckpt = aux ? (float*)(b + a.ckpt) : nullptr;
    p.F = a.F;
    return p;
}

// The same record read from global memory at a wave-uniform address: scalar loads straight into SGPRs
// (no LDS read, no v_readfirstlane per value).
__device__ __forceinline__ Rec read_rec_global(const float4* __restrict__ rec) {
    return rec_from_planes(rec[0], rec[1], rec[2], rec[3], rec[4], rec[5], rec[6], rec[7]);
}

// min over t in [lo, hi] of f(t) = |Q.xy + t A.xy|^2 - rm (Q.z + t A.z)^2 is <= 0?  (true when the slice
// is not convex in t: the conic is then not an ellipse there and nothing is culled)
__device__ __forceinline__ bool conic_edge(float ax, float ay, float az, float qx, float qy, float qz, float rm,
                                           float lo, float hi) {
    const float a = (ax * ax + ay * ay) - rm * (az * az);
    if (!(a > 0.0f)) return true;
    const float b = (qx * ax + qy * ay) - rm * (qz * az);
    const float t = fminf(fmaxf(-b / a, lo), hi);
    const float px = qx + t * ax, py = qy + t * ay, pz = qz + t * az;
    return (px * px + py * py) - rm * (pz * pz) <= 0.0f;
}

// Can splat j reach alpha >= 1/255 anywhere in the wave's block of pixel centres [wx0, wx1] x [wy0, wy1]?
// The homogeneous point is affine in the pixel offset d = pixel - anchor, p = d.x A + d.y B + (0, 0, Pz) (record
// planes 0-1), so the pair passes iff rho3 = |p.xy|^2 / p.z^2 <= rm = 2 ln(255 o) (or, with the AA filter, the
// disc 2 |pixel - centre|^2 <= rm): an ellipse (splats whose disc crosses the camera plane were culled
// upstream), tested exactly against the rectangle -- anchor inside, or an edge meeting it -- with a 1 %
// threshold margin and a 0.05 px larger rectangle, so the fp32 evaluation can never accept a pair the test
// rejected.
// (the cull fields are record dwords [0, 12): planes 0-2, RecField)
__device__ __forceinline__ bool may_hit_planes(float4 p0, float4 p1, float4 p2, float wx0, float wx1, float wy0,
                                               float wy1, bool aa) {
    const float v[12] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w, p2.x, p2.y, p2.z, p2.w};
    const float opac = fabsf(v[R_OPAC]);
    if (!(opac * 255.0f > 1.0f)) return false;
    const float rm = 2.0f * logf(255.0f * opac) * 1.01f + 1e-2f;
    const float x0 = wx0, x1 = wx1, y0 = wy0, y1 = wy1;  // (wave_block's cull box: already widened by 0.05)
    const float cx = v[R_XY], cy = v[R_XY + 1];
    if (aa) {
        const float ex = cx - fminf(fmaxf(cx, x0), x1), ey = cy - fminf(fmaxf(cy, y0), y1);
        if (2.0f * (ex * ex + ey * ey) <= rm) return true;
    }
    const float xa = v[R_XA], ya = v[R_YA];
    if (xa >= x0 && xa <= x1 && ya >= y0 && ya <= y1) return true;
    const float Ax = v[R_A], Ay = v[R_A + 1], Az = v[R_A + 2], Bx = v[R_B], By = v[R_B + 1], Bz = v[R_B + 2];
    const float Pz = v[R_PZ];
    const float dx0 = x0 - xa, dx1 = x1 - xa, dy0 = y0 - ya, dy1 = y1 - ya;
    return conic_edge(Ax, Ay, Az, dy0 * Bx, dy0 * By, Pz + dy0 * Bz, rm, dx0, dx1) ||
           conic_edge(Ax, Ay, Az, dy1 * Bx, dy1 * By, Pz + dy1 * Bz, rm, dx0, dx1) ||
           conic_edge(Bx, By, Bz, dx0 * Ax, dx0 * Ay, Pz + dx0 * Az, rm, dy0, dy1) ||
           conic_edge(Bx, By, Bz, dx1 * Ax, dx1 * Ay, Pz + dx1 * Az, rm, dy0, dy1);
}
template <int NB>
__device__ __forceinline__ bool wave_may_hit(const float4* s, int j, float wx0, float wx1, float wy0, float wy1,
                                             bool aa) {
    return may_hit_planes(s[0 * NB + j], s[1 * NB + j], s[2 * NB + j], wx0, wx1, wy0, wy1, aa);
}

struct Hit {
    float dx, dy, ipz, u, v, rho3, rho2, z, G, a_raw, alpha;
    f3 p;
    bool use3;
};

// reciprocal for values that feed no threshold decision (gradients and the distortion term only)
__device__ __forceinline__ float grad_rcp(float x) {
#if GSTEX_FAST_RCP
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}

// expf for x <= 0: the device library's expf sequence (two-part x*log2(e), rint, v_exp_f32, ldexp) without its
// overflow/underflow selects, so the same bits wherever expf is finite and non-zero.  The argument is
// clamped at -104 (expf's own flush-to-zero point; a NaN argument also lands there), so a degenerate
// pair gets G ~ 0 and fails the alpha test instead of propagating NaN.
__device__ __forceinline__ float exp_nonpos(float x) {
    x = fmaxf(x, -104.0f);
    const float ph = x * 1.44269502e+00f;                        // 0x3fb8aa3b
    float pl = __builtin_fmaf(x, 1.44269502e+00f, -ph);
    pl = __builtin_fmaf(x, 1.92596286e-08f, pl);                  // 0x32a5705f
    const float e = __builtin_rintf(ph);
    const float a = (ph - e) + pl;
    return __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(a), (int)e);
}

__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return __builtin_amdgcn_readfirstlane(v);
}
// The pair's offset from the anchor and homogeneous point p = k x l in affine form (gstex_common.h affine_homog):
// explicit fused multiply-adds (oracle/raster.py restates them: exact product, one rounding)
__device__ __forceinline__ void hit_p(const Rec& r, float px, float py, Hit& h) {
    h.dx = px - r.xa;
    h.dy = py - r.ya;
    h.p = f3{__builtin_fmaf(h.dx, r.A.x, h.dy * r.B.x), __builtin_fmaf(h.dx, r.A.y, h.dy * r.B.y),
             __builtin_fmaf(h.dy, r.B.z, __builtin_fmaf(h.dx, r.A.z, r.Pz))};
}
// The same for a near-edge-on splat (gstex_common.h kHpCos) from its fp64 setup row (A, B, Pz, anchor), each value
// rounded once: p is a small difference of larger terms there, and every value derived from it (u, v, the depth, the
// weights and all gradients through them) inherits the fp32 record's rounding amplified.  Used by every kernel that
// evaluates pairs of records carrying the mark (forward and backward alike, so both take the same decisions).
// The row is read with vector buffer loads (its 18 dwords would not fit beside the record in the kernels' SGPRs).
__device__ __forceinline__ double hp_load(__amdgpu_buffer_rsrc_t rs, int k) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, k * 8, 0, 0));
}
__device__ __forceinline__ void hit_p_hp(const double* __restrict__ row, float px, float py, Hit& h) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(row), 0, H_TW * 8,
                                                                        0x00020000);
    const double dx = (double)px - hp_load(rs, H_XA), dy = (double)py - hp_load(rs, H_YA);
    h.dx = (float)dx;
    h.dy = (float)dy;
    // one component at a time (the empty asm statements keep the row loads from being hoisted together): the
    // fp64 temporaries stay few, so the forward's visit loop keeps its register budget without spills
    h.p.x = (float)__builtin_fma(dx, hp_load(rs, H_A), dy * hp_load(rs, H_B));
    asm volatile("" : "+v"(h.p.x));
    h.p.y = (float)__builtin_fma(dx, hp_load(rs, H_A + 1), dy * hp_load(rs, H_B + 1));
    asm volatile("" : "+v"(h.p.y));
    h.p.z = (float)__builtin_fma(dy, hp_load(rs, H_B + 2), __builtin_fma(dx, hp_load(rs, H_A + 2), hp_load(rs, H_PZ)));
}
// The forward's copy: the row address is wave-uniform there, so plain loads become scalar loads and the row's
// doubles sit in SGPRs (fused multiply-adds take them as the scalar operand) -- the forward's visit loop is at its
// VGPR budget, and fp64 row values in VGPRs made the allocator spill the cull's loop-carried bounds
__device__ __forceinline__ void hit_p_hp_uniform(const double* __restrict__ row, float px, float py, Hit& h) {
    const double dx = (double)px - row[H_XA], dy = (double)py - row[H_YA];
    h.dx = (float)dx;
    h.dy = (float)dy;
    h.p = f3{(float)__builtin_fma(dx, row[H_A], dy * row[H_B]), (float)__builtin_fma(dx, row[H_A + 1], dy * row[H_B + 1]),
             (float)__builtin_fma(dy, row[H_B + 2], __builtin_fma(dx, row[H_A + 2], row[H_PZ]))};
}

// Returns false when the pair is skipped (degenerate, behind the near plane or alpha < 1/255).  h.dx, h.dy, h.p from
// hit_p / hit_p_hp.
__device__ __forceinline__ bool eval_rest(const Rec& r, float px, float py, bool aa, Hit& h) {
    // branch-free: a skipped pair's values are computed anyway (possibly inf/NaN) and never used, so
    // the callers see one predicate instead of three divergent exits (fewer exec-mask joins)
    const bool ok = h.p.z != 0.0f;
#if GSTEX_FAST_EVAL
    h.ipz = __builtin_amdgcn_rcpf(h.p.z);
#else
    h.ipz = 1.0f / h.p.z;
#endif
    h.u = h.p.x * h.ipz;
    h.v = h.p.y * h.ipz;
    h.rho3 = __builtin_fmaf(h.u, h.u, h.v * h.v);
    float dx = r.x - px, dy = r.y - py;
    h.rho2 = kFilterInvSq * __builtin_fmaf(dx, dx, dy * dy);
    h.use3 = !aa || (h.rho3 <= h.rho2);
    float rho = h.use3 ? h.rho3 : h.rho2;
    h.z = h.use3 ? __builtin_fmaf(h.u, r.Tw.x, __builtin_fmaf(h.v, r.Tw.y, r.Tw.z)) : r.Tw.z;
#if GSTEX_FAST_EVAL
    h.G = __builtin_amdgcn_exp2f(-0.72134752f * rho);  // exp(-rho/2) = 2^(-rho/(2 ln 2))
#else
    h.G = exp_nonpos(-0.5f * rho);
#endif
    h.a_raw = r.opac * h.G;
    h.alpha = fminf(kAlphaMax, h.a_raw);
    return ok && h.z >= kNear && h.alpha >= kAlphaMin;  // oracle/raster.py: nz & (zz >= near) & (alpha >= amin)
}
__device__ __forceinline__ bool eval_hit(const Rec& r, float px, float py, bool aa, Hit& h) {
    hit_p(r, px, py, h);
    return eval_rest(r, px, py, aa, h);
}

// One texel's channels: with C == 3 a single 12-B global_load_dwordx3 (the three channels share a cache
// line; three dword loads would look the same lines up three times in the vL1D).
struct __attribute__((aligned(4))) Texel3 { float v[3]; };
template <int CM>
__device__ __forceinline__ void load_texel(const float* __restrict__ p, int Cn, float (&out)[CM]) {
    if constexpr (CM == 3) {
        const Texel3 t = *reinterpret_cast<const Texel3*>(p);
        out[0] = t.v[0];
        out[1] = t.v[1];
        out[2] = t.v[2];
    } else {
#pragma unroll
        for (int c = 0; c < CM; ++c) out[c] = (c < Cn) ? p[c] : 0.0f;
    }
}

// A splat's texel block as a buffer resource: the wave-uniform block base and size live in SGPRs and
// each lane supplies a 32-bit byte offset, so a gather costs one buffer_load and no 64-bit address
// arithmetic; the hardware range check (size = the block's h*w*C floats) returns 0 outside the block.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t texel_rsrc(const float* texture, int off, int n_texels, int Cn) {
    off = __builtin_amdgcn_readfirstlane(off);
    n_texels = __builtin_amdgcn_readfirstlane(n_texels);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(texture) + (size_t)off * Cn, 0, n_texels * Cn * 4,
                                             0x00020000);
}
template <int CM>
__device__ __forceinline__ void load_texel_rs(__amdgpu_buffer_rsrc_t rs, int idx, int Cn, float (&out)[CM]) {
    if constexpr (CM == 3) {
        const auto t = __builtin_amdgcn_raw_buffer_load_b96(rs, idx * 12, 0, 0);
        out[0] = __int_as_float(t[0]);
        out[1] = __int_as_float(t[1]);
        out[2] = __int_as_float(t[2]);
    } else {
#pragma unroll
        for (int c = 0; c < CM; ++c)
            out[c] = (c < Cn) ? __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (idx * Cn + c) * 4, 0, 0)) : 0.0f;
    }
}

// The 4 bilinear texels of a splat block: byte offsets from one 24-bit multiply-add (v_mul_u32_u24 is
// full rate; the block index i*w + j < 2^24) plus wave-uniform row/column steps.
// Forward variant (C = 3): the far corners at i0 + 1 / j0 + 1 without the clamp to the block's edge.  When the
// coordinate is clamped to the last row / column its weight is exactly 0 (ax = 0 / ay = 0) and the lerp returns
// the near value bit for bit, so the far texel only has to be finite: one row down past the block reads 0 (buffer
// range check), one column right reads the next row's first texel.
__device__ __forceinline__ void load_texel_quad_unclamped(__amdgpu_buffer_rsrc_t rs, const Bilerp& b, int w,
                                                          float (&t00)[3], float (&t01)[3], float (&t10)[3],
                                                          float (&t11)[3]) {
    const int rowb = w * 12;  // row stride in bytes (wave-uniform: scalar when w is)
    const int o00 = (int)(__umul24(b.i0, (unsigned)rowb) + __umul24(b.j0, 12u));
    const int o10 = o00 + rowb;
    const auto a = __builtin_amdgcn_raw_buffer_load_b96(rs, o00, 0, 0);
    const auto c = __builtin_amdgcn_raw_buffer_load_b96(rs, o00 + 12, 0, 0);
    const auto d = __builtin_amdgcn_raw_buffer_load_b96(rs, o10, 0, 0);
    const auto e = __builtin_amdgcn_raw_buffer_load_b96(rs, o10 + 12, 0, 0);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        t00[k] = __int_as_float(a[k]);
        t01[k] = __int_as_float(c[k]);
        t10[k] = __int_as_float(d[k]);
        t11[k] = __int_as_float(e[k]);
    }
}
template <int CM>
__device__ __forceinline__ void load_texel_quad(__amdgpu_buffer_rsrc_t rs, const Bilerp& b, int w, int Cn,
                                                float (&t00)[CM], float (&t01)[CM], float (&t10)[CM],
                                                float (&t11)[CM]) {
    if constexpr (CM == 3) {
        const int o00 = (int)__umul24(__umul24(b.i0, w) + b.j0, 12u);
        const int o01 = b.j1 > b.j0 ? o00 + 12 : o00;
        const int o10 = b.i1 > b.i0 ? o00 + w * 12 : o00;
        const int o11 = b.j1 > b.j0 ? o10 + 12 : o10;
        const auto a = __builtin_amdgcn_raw_buffer_load_b96(rs, o00, 0, 0);
        const auto c = __builtin_amdgcn_raw_buffer_load_b96(rs, o01, 0, 0);
        const auto d = __builtin_amdgcn_raw_buffer_load_b96(rs, o10, 0, 0);
        const auto e = __builtin_amdgcn_raw_buffer_load_b96(rs, o11, 0, 0);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            t00[k] = __int_as_float(a[k]);
            t01[k] = __int_as_float(c[k]);
            t10[k] = __int_as_float(d[k]);
            t11[k] = __int_as_float(e[k]);
        }
    } else if constexpr (CM == 6) {
        // the eval render's 6 channels: two 12-B loads per corner (24 B contiguous per texel) instead of six dwords
        const int o00 = (int)__umul24(__umul24(b.i0, w) + b.j0, 24u);
        const int o01 = b.j1 > b.j0 ? o00 + 24 : o00;
        const int o10 = b.i1 > b.i0 ? o00 + w * 24 : o00;
        const int o11 = b.j1 > b.j0 ? o10 + 24 : o10;
        const int off[4] = {o00, o01, o10, o11};
        float (*dst[4])[CM] = {&t00, &t01, &t10, &t11};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const auto lo = __builtin_amdgcn_raw_buffer_load_b96(rs, off[q], 0, 0);
            const auto hi = __builtin_amdgcn_raw_buffer_load_b96(rs, off[q] + 12, 0, 0);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                (*dst[q])[k] = __int_as_float(lo[k]);
                (*dst[q])[3 + k] = __int_as_float(hi[k]);
            }
        }
    } else {
        load_texel_rs<CM>(rs, b.i0 * w + b.j0, Cn, t00);
        load_texel_rs<CM>(rs, b.i0 * w + b.j1, Cn, t01);
        load_texel_rs<CM>(rs, b.i1 * w + b.j0, Cn, t10);
        load_texel_rs<CM>(rs, b.i1 * w + b.j1, Cn, t11);
    }
}

// the sample point in texel units (xr, yr) = (tu h, tv w) from the record's prescaled texture affine (setup_kernel)
__device__ __forceinline__ void tex_coords(const Rec& r, float u, float v, float& xr, float& yr) {
    xr = __builtin_fmaf(u, r.auu, __builtin_fmaf(v, r.auv, r.tu0));  // fused (oracle/raster.py restates it)
    yr = __builtin_fmaf(u, r.avu, __builtin_fmaf(v, r.avv, r.tv0));
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
// acc + w (tex_scale * bilinear(v) + tex_bias) in lerp form with fused multiply-adds (8 VALU per channel instead of
// 13): no threshold decision depends on a texel value, so it is compared with the oracle within tolerance only
__device__ __forceinline__ float tex_accum(float acc, float v00, float v01, float v10, float v11, float ax, float ay,
                                           float s, float b, float w) {
    const float top = __builtin_fmaf(ay, v01 - v00, v00);
    const float bot = __builtin_fmaf(ay, v11 - v10, v10);
    const float mix = __builtin_fmaf(ax, bot - top, top);
    return __builtin_fmaf(__builtin_fmaf(mix, s, b), w, acc);
}
// GEOF = false: depth / distortion / normal not produced (their outputs are NULL: a caller whose loss does
// not use them, e.g. the photometric training step); every other output is computed unchanged.
// One 256-thread workgroup per tile; its four quadrant waves share 128-record batches staged in LDS (a barrier per
// batch).  (One wave64 workgroup per (tile, quadrant) with scalar record loads measured 12 % slower in round 3: the
// shared staging reads each record once per tile instead of once per quadrant.)
template <int C, bool GEOF>
__global__ __launch_bounds__(kThreads, GSTEX_FWD_OCC) void raster_fwd_kernel(
    CamArgs cam_args, int tiles_x, int settings, const float* __restrict__ bg, int Cdyn,
    const float4* __restrict__ records, const double* __restrict__ hp_records, const int2* __restrict__ tile_ranges,
    const int32_t* __restrict__ tile_order,
    const int32_t* __restrict__ sorted_ids, const float* __restrict__ texture, int n_texels, float tex_scale,
    float tex_bias, float* __restrict__ out_img,
    float* __restrict__ out_depth, float* __restrict__ out_reg, float* __restrict__ out_alpha,
    float* __restrict__ out_tex, float* __restrict__ out_normal, float4* __restrict__ state, AuxPtrs aux,
    int n_tiles, const ZeroBufs zb) {
    const Camera cam = load_camera(cam_args);
    unsigned long long* __restrict__ visit_masks = aux.masks;
    zero_bufs(zb);
    constexpr int CM = (C > 0) ? C : 8;  // register capacity for the runtime-C path
    const int Cn = (C > 0) ? C : Cdyn;
    constexpr int kStep = kFwdBatch, kWords = kStep / 64;
    __shared__ float4 s_rec[kRecF4 * kFwdBatch];
    __shared__ int s_gid[kFwdBatch];  // the batch's splat ids (the near-edge-on splats' fp64 rows are read by id)
    // the next batch's ids, copied global -> LDS (no VGPR) during the current batch's visits, so the batch staging's
    // record loads do not wait on a dependent id load first (raster loop at cfg3: forward 0.510 vs 0.5155 ms)
    __shared__ int s_gid_next[kFwdBatch];
    const int ti = (int)blockIdx.x;
    const int tile = tile_order ? tile_order[ti] : ti;  // largest-first when given
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    const int tid = (int)threadIdx.x;
    const WaveBlock wb = wave_block(tx, ty, tid);
    const int pxi = wb.px, pyi = wb.py;
    const bool inside = pxi < cam.W && pyi < cam.H;
    const float px = (float)pxi + 0.5f, py = (float)pyi + 0.5f;  // pixel centres (gstex_common.h)
    const bool aa = (settings & GSTEX_SETTING_AA_BLUR) != 0;
    const bool dreg = (settings & GSTEX_SETTING_DIST_REG) != 0;
    const int2 rng = tile_ranges[tile];
    const float bg0 = bg ? bg[0] : 0.f, bg1 = bg ? bg[1] : 0.f, bg2 = bg ? bg[2] : 0.f;
    const float wx0 = wb.wx0, wx1 = wb.wx1, wy0 = wb.wy0, wy1 = wb.wy1;

    float T = 1.0f;
    float img[3] = {0.f, 0.f, 0.f}, nrm[3] = {0.f, 0.f, 0.f};
    float tex[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c) tex[c] = 0.f;
    float D = 0.f, M1 = 0.f, M2 = 0.f, reg = 0.f;
    int last = -1;
    // per-lane "still running" as a float, not a bool: a bool carried around the visit loop becomes an SGPR lane
    // mask that the compiler re-merges with exec at every join (three SALU per join; measured: the forward with the
    // divergent per-lane loop exits and bool lane state 0.595 ms, with this loop 0.550 ms)
    float alive = inside ? 1.0f : 0.0f;
#define GSTEX_FWD_DONE (alive == 0.0f)
    // Deferred texel accumulation (kFwdDefer): a visit's four texel gathers are issued into the pending registers
    // and folded into tex[] at the lane's next contributing visit (or at a checkpoint / the end), so their latency
    // overlaps the next visit's record read and pair evaluation.  Same values, same order of accumulation.
    constexpr bool kDefer = kFwdDefer && C == 3;
    float pend = 0.0f;  // (a float: see `alive`)
    float p00[CM], p01[CM], p10[CM], p11[CM], pax = 0.f, pay = 0.f, pw = 0.f;
    // kDefer: tex[c] accumulates sum_k w_k bilerp_k(texels) with the weight folded into the four corner weights (4
    // fused multiply-adds per channel), texw = sum_k w_k over the textured visits, and the affine (tex_scale, tex_bias)
    // is applied once, by tex_value(): sum_k w_k (s m_k + b) = s sum_k w_k m_k + b sum_k w_k (9 + 4 C VALU per visit
    // instead of 8 C; no decision depends on a texel value)
    float texw = 0.0f;
    auto fold_set = [&](float (&a00)[CM], float (&a01)[CM], float (&a10)[CM], float (&a11)[CM], float ax, float ay,
                        float aw, float& apend) {
        if (kDefer && apend != 0.0f) {
            const float c1 = aw * ax, c0 = aw * (1.0f - ax), qy = 1.0f - ay;
            const float w00 = c0 * qy, w01 = c0 * ay, w10 = c1 * qy, w11 = c1 * ay;
#pragma unroll
            for (int c = 0; c < CM; ++c) {
                if (c < Cn)
                    tex[c] = __builtin_fmaf(a11[c], w11, __builtin_fmaf(a10[c], w10, __builtin_fmaf(a01[c], w01,
                             __builtin_fmaf(a00[c], w00, tex[c]))));
            }
            texw = texw + aw;
            apend = 0.0f;
        }
    };
    auto fold_pending = [&]() { fold_set(p00, p01, p10, p11, pax, pay, pw, pend); };
    auto tex_value = [&](int c) {  // the texture output of channel c so far
        return kDefer ? __builtin_fmaf(tex[c], tex_scale, tex_bias * texw) : tex[c];
    };
    const int lane = tid & 63, wave = tid >> 6;
    const size_t vm_base = visit_mask_base(rng.x, tile);
    const int sbase = seg_base(rng.x, tile);
    int seg_visits = 0, cur_seg = 0;  // this wave's splat evaluations in the current segment (backward cost)
    // XCD group of the tile's backward units: its GSTEX_XCD_MB x GSTEX_XCD_MB-tile macro-block
    const int xgroup = (((tx / GSTEX_XCD_MB) + (ty / GSTEX_XCD_MB) * ((tiles_x + GSTEX_XCD_MB - 1) / GSTEX_XCD_MB)) & 7)
                       << 24;
    if (aux.slot_tile)
        for (int k = tid; k * kSegLen < rng.y - rng.x; k += kThreads) aux.slot_tile[sbase + k] = tile;
    // one checkpoint record: field f of the wave's lane at ckpt[((slot * 4 + wave) * F + f) * 64 + lane]
    auto write_ck = [&](int slot) {
        float* ck = aux.ckpt + ((size_t)slot * 4 + wave) * aux.F * 64 + lane;
        ck[0] = T;
        ck[64] = img[0];
        ck[128] = img[1];
        ck[192] = img[2];
#pragma unroll
        for (int c = 0; c < CM; ++c)
            if (c < Cn) ck[(4 + c) * 64] = tex_value(c);
        if (GEOF) {
            float* g = ck + (4 + Cn) * 64;
            g[0] = D;
            g[64] = nrm[0];
            g[128] = nrm[1];
            g[192] = nrm[2];
            g[256] = M1;
            g[320] = M2;
        }
    };

    if (tid < kFwdBatch && rng.x + tid < rng.y) s_gid_next[tid] = sorted_ids[rng.x + tid];  // the first batch's
    for (int b0 = rng.x; b0 < rng.y; b0 += kStep) {
        if (aux.cost && b0 > rng.x && (b0 - rng.x) % kSegLen == 0) {
            // segment cur_seg complete: its cost, and the state after it while a lane of the wave still runs
            const int cnt = wave_max_i(seg_visits);  // lanes leave the visit loop as they finish: the wave's count
            if (lane == 0 && cnt) {
                const int key = ((cnt >> GSTEX_UNIT_COARSE) + 1) | xgroup;
                aux.cost[(sbase + cur_seg) * 4 + wave] = key;
                atomicAdd(&aux.order_ws[unit_bin(key)], 1);  // the backward's unit-order histogram
            }
            fold_pending();
            if (__any(!GSTEX_FWD_DONE)) write_ck(sbase + cur_seg);
            seg_visits = 0;
            ++cur_seg;
        }
        const int nb = min(kStep, rng.y - b0);
        if (__syncthreads_count(GSTEX_FWD_DONE ? 1 : 0) == kThreads) break;
        for (int q = tid; q < kFwdBatch * kRecF4; q += kThreads) {
            const int j = q / kRecF4, k = q % kRecF4;
            if (b0 + j < rng.y) {
                const int gid = s_gid_next[j];
                s_rec[k * kFwdBatch + j] = records[(size_t)gid * kRecF4 + k];
                if (k == 0) s_gid[j] = gid;
            }
        }
        __syncthreads();
        if (tid < kFwdBatch && b0 + kStep < rng.y) {  // waves 0-1: lane l of wave w fetches id kStep + 64 w + l ahead
            const int nx = min(b0 + kStep + tid, rng.y - 1);  // (past the list: a valid address, value unused)
            __builtin_amdgcn_global_load_lds(const_cast<int32_t*>(sorted_ids + nx), s_gid_next + (tid & ~63), 4, 0, 0);
        }
        // the batch splats whose contribution region meets this wave's 8x8 block, tested all at once
        unsigned long long todo[kWords];
#pragma unroll
        for (int hb = 0; hb < kWords; ++hb) {
            const int jj = hb * 64 + lane;
            const bool hit = jj < nb && wave_may_hit<kFwdBatch>(s_rec, jj < nb ? jj : 0, wx0, wx1, wy0, wy1, aa);
            todo[hb] = __ballot(hit);
            GSTEX_STAT(8, (unsigned long long)max(0, min(64, nb - hb * 64)));  // cull candidates (wave, splat)
            GSTEX_STAT(9, __popcll(todo[hb]));                                 // passing the wave's cull
            // hand the cull to the backward, which visits these splats up to the wave's last contributor
            if (visit_masks && lane == 0 && hb * 64 < nb)
                visit_masks[(vm_base + ((b0 - rng.x) >> 6) + hb) * 4 + wave] = todo[hb];
        }
        // wave-uniform visit loop: finished lanes stay in it with their updates predicated off (no divergent exits:
        // the loop control is a scalar bit scan, not exec-mask bookkeeping); it ends when the batch's bits run out
        // or every lane of the wave has finished
        bool all_done = __all(GSTEX_FWD_DONE);
        for (int hb = 0; hb < kWords && !all_done; ++hb) {
          unsigned long long m = todo[hb];
          while (m) {
            const int j = hb * 64 + __builtin_ctzll(m);
            m &= m - 1;
            const Rec r = read_rec<kFwdBatch>(s_rec, j);
            ++seg_visits;
            Hit h;
            hit_p(r, px, py, h);
            // a near-edge-on splat (the record opacity's sign bit, wave-uniform): p from its fp64 row
            if (hp_records && __builtin_amdgcn_readfirstlane(__float_as_int(r.mark)) < 0)
                hit_p_hp_uniform(hp_records + (size_t)__builtin_amdgcn_readfirstlane(s_gid[j]) * H_FIELDS, px, py, h);
            const bool ok = eval_rest(r, px, py, aa, h) && alive != 0.0f;
            const float test_T = T * (1.0f - h.alpha);
            const bool stop = ok && test_T < kTMin;
            GSTEX_STAT(10, 1);                                    // visits (the wave evaluates a splat)
            GSTEX_STAT(11, __ballot(ok) ? 1 : 0);                 // ... with a contributing lane
            GSTEX_STAT(12, __popcll(__ballot(ok && !stop)));      // contributing lanes
            alive = stop ? 0.0f : alive;
            if (ok && !stop) {
                const float w = h.alpha * T;
                const int bh = __builtin_amdgcn_readfirstlane(r.h), bw = __builtin_amdgcn_readfirstlane(r.w);
                const int boff = __builtin_amdgcn_readfirstlane(r.off);
                const bool has_tex = bh * bw > 0 && boff + bh * bw <= n_texels;
                if (kDefer) {
                    // (computed whether or not the splat has texels: used only when it has)
                    float tu, tv;
                    tex_coords(r, h.u, h.v, tu, tv);
                    const Bilerp b = bilerp_xy(tu, tv, bh, bw, r.hm1, r.wm1);
                    fold_pending();
                    if (has_tex) {
                        const __amdgpu_buffer_rsrc_t rs = texel_rsrc(texture, boff, bh * bw, Cn);
                        if constexpr (CM == 3) load_texel_quad_unclamped(rs, b, bw, p00, p01, p10, p11);
                        else load_texel_quad<CM>(rs, b, bw, Cn, p00, p01, p10, p11);
                        pax = b.ax;
                        pay = b.ay;
                        pw = w;
                        pend = 1.0f;
                    }
                } else if (has_tex) {
                    float tu, tv;
                    tex_coords(r, h.u, h.v, tu, tv);
                    const Bilerp b = bilerp_xy(tu, tv, r.h, r.w, r.hm1, r.wm1);
                    const __amdgpu_buffer_rsrc_t rs = texel_rsrc(texture, boff, bh * bw, Cn);
                    float t00[CM], t01[CM], t10[CM], t11[CM];
                    load_texel_quad<CM>(rs, b, bw, Cn, t00, t01, t10, t11);
#pragma unroll
                    for (int c = 0; c < CM; ++c)
                        if (c < Cn) tex[c] = tex_accum(tex[c], t00[c], t01[c], t10[c], t11[c], b.ax, b.ay, tex_scale, tex_bias, w);
                }
                img[0] = __builtin_fmaf(r.rgb[0], w, img[0]);
                img[1] = __builtin_fmaf(r.rgb[1], w, img[1]);
                img[2] = __builtin_fmaf(r.rgb[2], w, img[2]);
                if (GEOF) {
                    D = D + h.z * w;
                    nrm[0] = nrm[0] + r.nrm[0] * w;
                    nrm[1] = nrm[1] + r.nrm[1] * w;
                    nrm[2] = nrm[2] + r.nrm[2] * w;
                }
                if (GEOF && dreg) {
                    const float A = 1.0f - T;
                    const float mm = kFarRatio * (1.0f - kNear * grad_rcp(h.z));
                    reg = reg + ((mm * mm * A + M2) - 2.0f * mm * M1) * w;
                    M1 = M1 + mm * w;
                    M2 = M2 + mm * mm * w;
                }
                T = test_T;
                last = b0 - rng.x + j;
            }
            if (__builtin_amdgcn_ballot_w64(alive != 0.0f) == 0) {
                all_done = true;
                break;
            }
          }
        }
    }
    fold_pending();
    if (aux.cost) {
        const int cnt = wave_max_i(seg_visits);
        if (lane == 0 && cnt) {
            const int key = ((cnt >> GSTEX_UNIT_COARSE) + 1) | xgroup;
            aux.cost[(sbase + cur_seg) * 4 + wave] = key;
            atomicAdd(&aux.order_ws[unit_bin(key)], 1);
        }
        // final accumulators for the backward's earlier segments, in the slot of the wave's last segment
        const int wl = wave_max_i(last);
        if (wl >= kSegLen) write_ck(sbase + wl / kSegLen);
    }
    if (!inside) return;
    const size_t pix = (size_t)pyi * cam.W + pxi;
    out_img[3 * pix + 0] = img[0] + T * bg0;
    out_img[3 * pix + 1] = img[1] + T * bg1;
    out_img[3 * pix + 2] = img[2] + T * bg2;
    if (GEOF) {
        out_depth[pix] = D;
        out_reg[pix] = reg;
    }
    out_alpha[pix] = 1.0f - T;
#pragma unroll
    for (int c = 0; c < CM; ++c)
        if (c < Cn) out_tex[(size_t)Cn * pix + c] = tex_value(c);
    if (GEOF) {
        if (settings & GSTEX_SETTING_EVAL_NORMAL) {
            // bit 15 (gstex.py:1198-1203, the eval "clean normal" render): the accumulated normal is returned
            // as a unit vector (0 where nothing was accumulated); every other output is unchanged
            const float n2 = (nrm[0] * nrm[0] + nrm[1] * nrm[1]) + nrm[2] * nrm[2];
            const float inv = n2 > 0.0f ? 1.0f / sqrtf(n2) : 0.0f;
            nrm[0] = nrm[0] * inv;
            nrm[1] = nrm[1] * inv;
            nrm[2] = nrm[2] * inv;
        }
        out_normal[3 * pix + 0] = nrm[0];
        out_normal[3 * pix + 1] = nrm[1];
        out_normal[3 * pix + 2] = nrm[2];
    }
    state[pix] = make_float4(T, M1, M2, __int_as_float(last));
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------
// Reduce-scatter butterfly over the 64 lanes, entirely on VALU cross-lane ops (no LDS traffic):
// xor-32 and xor-16 halvings with v_permlane32_swap / v_permlane16_swap, xor-8 with DPP row_ror:8,
// then an 8-lane all-reduce (quad_perm xor1, xor2, row_half_mirror).  On return, lane l with
// (l & 7) == 0 holds the wave sums of values [NV/2 b5 + NV/4 b4 + NV/8 b3 + 0 .. NV/8 - 1] (b5,b4,b3 = bits of l).
template <int NV>
__device__ __forceinline__ void wave_reduce(float (&v)[NV]) {
    static_assert(NV == 24 || NV == 32, "reduce-scatter over 8 lane groups of 3 or 4 values");
    constexpr int H = NV / 2, Q = NV / 4, E = NV / 8;
    const int lane = threadIdx.x & 63;
    // permlane32_swap(a, b) leaves a = [a_lo, b_lo], b = [a_hi, b_hi]: a + b holds a's half-sum in
    // lanes 0-31 and b's in lanes 32-63 (likewise per row pair for permlane16_swap)
#pragma unroll
    for (int i = 0; i < H; ++i) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i + H]), false, false);
        v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
#pragma unroll
    for (int i = 0; i < Q; ++i) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i + Q]), false, false);
        v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    {
        // the last four stages as single v_add_f32_dpp instructions (the compiler emits a DPP move plus an add):
        // row_ror:8 (lane ^ 8 inside a 16-lane row), quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror (the other
        // quad of the 8-lane group).  dpp(x) + y rounds as y + dpp(x).  The leading s_nop covers the VALU-write ->
        // DPP-read hazard for the inputs (the asm is opaque to the hazard recognizer); inside, each value is DPP-read
        // again only after the other E - 1 >= 2 values' writes; the trailing s_nop covers a following DPP read.
        const bool hi = lane & 8;
        float keep[4], send[4];
#pragma unroll
        for (int i = 0; i < E; ++i) {
            send[i] = hi ? v[i] : v[i + E];
            keep[i] = hi ? v[i + E] : v[i];
        }
#define GSTEX_DPP_ADD(CTRL, D, S) "v_add_f32_dpp %" #D ", %" #S ", %" #D " " CTRL " row_mask:0xf bank_mask:0xf\n"
#define GSTEX_DPP_SELF(CTRL, D) "v_add_f32_dpp %" #D ", %" #D ", %" #D " " CTRL " row_mask:0xf bank_mask:0xf\n"
        if constexpr (E == 3) {
            asm volatile("s_nop 1\n"
                         GSTEX_DPP_ADD("row_ror:8", 0, 3) GSTEX_DPP_ADD("row_ror:8", 1, 4) GSTEX_DPP_ADD("row_ror:8", 2, 5)
                         GSTEX_DPP_SELF("quad_perm:[1,0,3,2]", 0) GSTEX_DPP_SELF("quad_perm:[1,0,3,2]", 1)
                         GSTEX_DPP_SELF("quad_perm:[1,0,3,2]", 2)
                         GSTEX_DPP_SELF("quad_perm:[2,3,0,1]", 0) GSTEX_DPP_SELF("quad_perm:[2,3,0,1]", 1)
                         GSTEX_DPP_SELF("quad_perm:[2,3,0,1]", 2)
                         GSTEX_DPP_SELF("row_half_mirror", 0) GSTEX_DPP_SELF("row_half_mirror", 1)
                         GSTEX_DPP_SELF("row_half_mirror", 2)
                         "s_nop 1"
                         : "+v"(keep[0]), "+v"(keep[1]), "+v"(keep[2])
                         : "v"(send[0]), "v"(send[1]), "v"(send[2]));
        } else {
            asm volatile("s_nop 1\n"
                         GSTEX_DPP_ADD("row_ror:8", 0, 4) GSTEX_DPP_ADD("row_ror:8", 1, 5) GSTEX_DPP_ADD("row_ror:8", 2, 6)
                         GSTEX_DPP_ADD("row_ror:8", 3, 7)
                         GSTEX_DPP_SELF("quad_perm:[1,0,3,2]", 0) GSTEX_DPP_SELF("quad_perm:[1,0,3,2]", 1)
                         GSTEX_DPP_SELF("quad_perm:[1,0,3,2]", 2) GSTEX_DPP_SELF("quad_perm:[1,0,3,2]", 3)
                         GSTEX_DPP_SELF("quad_perm:[2,3,0,1]", 0) GSTEX_DPP_SELF("quad_perm:[2,3,0,1]", 1)
                         GSTEX_DPP_SELF("quad_perm:[2,3,0,1]", 2) GSTEX_DPP_SELF("quad_perm:[2,3,0,1]", 3)
                         GSTEX_DPP_SELF("row_half_mirror", 0) GSTEX_DPP_SELF("row_half_mirror", 1)
                         GSTEX_DPP_SELF("row_half_mirror", 2) GSTEX_DPP_SELF("row_half_mirror", 3)
                         "s_nop 1"
                         : "+v"(keep[0]), "+v"(keep[1]), "+v"(keep[2]), "+v"(keep[3])
                         : "v"(send[0]), "v"(send[1]), "v"(send[2]), "v"(send[3]));
        }
#undef GSTEX_DPP_ADD
#undef GSTEX_DPP_SELF
#pragma unroll
        for (int i = 0; i < E; ++i) v[i] = keep[i];
    }
}

// ------------------------------------------------------------------------------------------
// texel-gradient pre-reduction: along each 16-lane row (16 consecutive pixels of one image row)
// the bilinear cell of a splat's texture forms contiguous runs, so a segmented inclusive scan
// by cell key with DPP row shifts leaves each run's sum in its last lane; only run tails issue
// the 4*C atomics (instead of every contributing lane, which serialised on the LDS atomic unit).
// ------------------------------------------------------------------------------------------
// row_shr:OFF with out-of-row lanes reading 0 (bound_ctrl)
template <int CTRL>
__device__ __forceinline__ int dpp_bc_i(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
template <int OFF>
__device__ __forceinline__ float dpp_shr_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x110 + OFF, 0xF, 0xF, false));
}

// v += row_shr:OFF(v) * mf, mf = 1 where the lane OFF to the left is in the same segment, else 0: one
// v_fmac_f32 with a DPP source per value (the compiler does not fold a DPP move into the tied-accumulator
// fmac, so it is written out).  fma(t, 1, v) rounds as t + v and fma(t, 0, v) = v, so the result equals the
// add-and-select form bit for bit.  The leading s_nop covers the VALU-write -> DPP-read hazard for the
// values' last writers (the asm is opaque to the compiler's hazard recognizer); within the block each value is
// read by DPP only after the other NV - 1 writes, and the trailing s_nop covers the compiler's next DPP read.
template <int OFF>
__device__ __forceinline__ void fmac_dpp_shr(float& v, float mf) {
    if constexpr (OFF == 1)
        asm volatile("v_fmac_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v) : "v"(mf));
    else if constexpr (OFF == 2)
        asm volatile("v_fmac_f32_dpp %0, %0, %1 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v) : "v"(mf));
    else if constexpr (OFF == 4)
        asm volatile("v_fmac_f32_dpp %0, %0, %1 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v) : "v"(mf));
    else
        asm volatile("v_fmac_f32_dpp %0, %0, %1 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v) : "v"(mf));
}
// Segments = maximal runs of equal key inside a 16-lane row (a lane whose key differs from its left
// neighbour starts a segment, so a non-contributing lane splits a run instead of being bridged).
// Returns true for the last lane of a segment with key >= 0; it then holds the segment's sums.
// 1.0f in the lanes whose bit of the wave mask m is set, else 0 (one v_cndmask with the mask as lane select)
__device__ __forceinline__ float mask_one(unsigned long long m) {
    float r;
    asm("v_cndmask_b32_e64 %0, 0, 1.0, %1" : "=v"(r) : "s"(m));
    return r;
}
// The segment heads as one wave mask H (ballot of key changes, plus every group's first
// lane); lane l joins lane l - OFF iff no head lies in (l - OFF, l], i.e. bit l of ~(H | H << 1 | ... | H << (OFF-1)),
// computed on the scalar unit; the run tails are the lanes before a head or at a group's end.
template <int NV>
__device__ __forceinline__ bool seg_reduce_rows(int key, float (&v)[NV]) {
    constexpr int SW = GSTEX_SEG_W;
    static_assert(SW == 2 || SW == 4 || SW == 8 || SW == 16, "segment width");
    constexpr unsigned long long kFirst = SW == 2 ? 0x5555555555555555ull : SW == 4 ? 0x1111111111111111ull
                                        : SW == 8 ? 0x0101010101010101ull : 0x0001000100010001ull;
    constexpr unsigned long long kLast = kFirst << (SW - 1);
    const int left = dpp_bc_i<0x111>(key);  // row_shr:1 (lanes at a group start are heads regardless)
    const unsigned long long H = __ballot(left != key) | kFirst;
    const unsigned long long live = __ballot(key >= 0);
    unsigned long long cover = H;  // heads in (l - off, l] for the current off
#pragma unroll
    for (int off = 1; off < SW; off <<= 1) {
        const float mf = mask_one(~cover);
        asm volatile("s_nop 1" ::: "memory");
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            if (off == 1) fmac_dpp_shr<1>(v[i], mf);
            else if (off == 2) fmac_dpp_shr<2>(v[i], mf);
            else if (off == 4) fmac_dpp_shr<4>(v[i], mf);
            else fmac_dpp_shr<8>(v[i], mf);
        }
        asm volatile("s_nop 1" ::: "memory");
        cover = cover | (cover << off);
    }
    const unsigned long long tails = ((H >> 1) | kLast) & live;
    return mask_one(tails) != 0.0f;
}

// Backward: one wave64 workgroup per (tile, 8x8 quadrant) -- the 4 quadrant waves of a tile share nothing, so
// no wave ever waits for another (no barriers; a finished wave frees its slot at once).  The wave walks the
// tile list back to front over the forward's cull bits for its quadrant, up to its last contributor.  Per
// visited splat it reduces its 24 gradient partials across its 64 pixels and adds them into the splat's accumulator
// row with one float-atomic instruction; in the deterministic mode (row_flags given) it stores them instead as the
// (pair, quadrant) row partials[slot][quadrant] (slot = the pair's emission slot), flagging the row in
// row_flags[slot] (byte = quadrant; rows never written stay unflagged and are never read), and
// gstex_raster_setup_bwd sums each splat's flagged rows in (slot, quadrant) order -> bitwise reproducible.
// Texel gradients: segmented scan along each 4-pixel half row, run tails
// added to the splat's texel block staged in the wave's LDS as int32 fixed point (exact, order-independent),
// and the block flushed to v_texture (global float atomics, non-zero entries only) right after the visit.
//
// GEO = false: no depth / distortion / normal upstream gradient (all NULL, the training default:
// gstex.py:198-201 sets both weights to 0), so every term they scale is dropped at compile time.  The
// remaining arithmetic is unchanged (x + 0 * y = x), so both variants give the same values.

// Texel-gradient fixed point, per visit: the reduce also sums M = sum over the wave's pixels of |w tex_scale| x
// max_c |dL/dtex[c]|, a bound on what the visit adds to any staged entry (bilinear weights <= 1).  Contributions
// are formed at scale 2^S, S = 30 - e (M < 2^e); each run tail of the 8-lane row scan (< 2^30) is rounded to
// int32 (one v_cvt_rpi_i32_f32) and the tails are summed exactly in int32 (|sum| <= 2^30 + rounding).
// Resolution: 2^-30 of the visit's total.
__device__ __forceinline__ int fixed_round(float y) {  // y already scaled by 2^S; round half up, one VALU op
    int q;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(q) : "v"(y));
    return q;
}
constexpr int kTexFixBits = 30;

// (fp32 staging with ds_add_f32 instead measured 2x slower: 3.2 vs 1.57 ms, round 2; 3.0 vs 1.4 ms, round 4)
__device__ __forceinline__ void stage_add(int* a, float y) { atomicAdd(a, fixed_round(y)); }
#ifndef GSTEX_FLUSH_U
#define GSTEX_FLUSH_U 4
#endif
constexpr int kFlushU = GSTEX_FLUSH_U;  // staging entries per lane per flush pass
static_assert(kTexStage % (64 * kFlushU) == 0, "flush passes tile the staging area");


template <int C, bool GEO>
__global__ __launch_bounds__(64, (BwdShape<C, GEO>::kWaves)) void raster_bwd_kernel(
    CamArgs cam_args, int tiles_x, int settings, const float* __restrict__ bg, int Cdyn,
    const float4* __restrict__ records, const double* __restrict__ hp_records, const int2* __restrict__ tile_ranges,
    const int32_t* __restrict__ sorted_ids, const int32_t* __restrict__ sorted_slots, const float* __restrict__ texture,
    int n_texels, float tex_scale, float tex_bias, const float4* __restrict__ state, const float* __restrict__ v_img,
    const float* __restrict__ v_depth, const float* __restrict__ v_reg, const float* __restrict__ v_alpha,
    const float* __restrict__ v_tex, const float* __restrict__ v_normal, float* __restrict__ partials,
    unsigned char* __restrict__ row_flags, float* __restrict__ v_texture, const AuxPtrs aux, const ZeroBufs zb) {
    zero_bufs(zb);
    const Camera cam = load_camera(cam_args);
    constexpr int CM = (C > 0) ? C : 8;
    const int Cn = (C > 0) ? C : Cdyn;
    __shared__ int s_texq[kTexStage];

    // unit = 4 slot + quadrant (see AuxPtrs), launched costliest first; a unit the forward never evaluated in is empty
    const int unit = aux.order[blockIdx.x] - 1;  // entries are unit + 1
    if (unit < 0) return;  // a launch position no unit was placed at (empty units take none)
    const int quad = unit & 3, slot = unit >> 2;
    const int tile = aux.slot_tile[slot];
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    const int lane = threadIdx.x;
    const WaveBlock wb = wave_block(tx, ty, quad * 64 + lane);
    const int pxi = wb.px, pyi = wb.py;
    const bool inside = pxi < cam.W && pyi < cam.H;
    const float px = (float)pxi + 0.5f, py = (float)pyi + 0.5f;  // pixel centres (gstex_common.h)
    const bool aa = (settings & GSTEX_SETTING_AA_BLUR) != 0;
    const bool dreg = (settings & GSTEX_SETTING_DIST_REG) != 0;
    const int2 rng = tile_ranges[tile];
    const float bg0 = bg ? bg[0] : 0.f, bg1 = bg ? bg[1] : 0.f, bg2 = bg ? bg[2] : 0.f;

    float T = 1.0f, M1f = 0.f, M2f = 0.f;
    int last = -1;
    float Gimg[3] = {0.f, 0.f, 0.f}, Gn[3] = {0.f, 0.f, 0.f}, Gtex[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c) Gtex[c] = 0.f;
    float Gd = 0.f, Greg = 0.f, Ga = 0.f;
    if (inside) {
        const size_t pix = (size_t)pyi * cam.W + pxi;
        const float4 st = state[pix];
        T = st.x; M1f = st.y; M2f = st.z; last = __float_as_int(st.w);
        // a NULL upstream gradient (an output the loss does not use) counts as zero
        if (v_img) { Gimg[0] = v_img[3 * pix]; Gimg[1] = v_img[3 * pix + 1]; Gimg[2] = v_img[3 * pix + 2]; }
#pragma unroll
        for (int c = 0; c < CM; ++c)
            if (c < Cn && v_tex) Gtex[c] = v_tex[(size_t)Cn * pix + c];
        Ga = v_alpha ? v_alpha[pix] : 0.f;
        if (GEO) {
            Gd = v_depth ? v_depth[pix] : 0.f;
            Greg = (dreg && v_reg) ? v_reg[pix] : 0.f;
            if (v_normal) { Gn[0] = v_normal[3 * pix]; Gn[1] = v_normal[3 * pix + 1]; Gn[2] = v_normal[3 * pix + 2]; }
        }
    }
    // the wave's last contributor: pairs behind it receive no gradient from this quadrant (no row, no flag); this
    // unit walks tile-list positions [lo, hi] of its segment
    const int wave_last = wave_max_i(last);
    GSTEX_WG_STAMP(rng.y - rng.x, wave_last);
    const int sbase = seg_base(rng.x, tile);
    const int seg = slot - sbase, lo = seg * kSegLen;
    if (wave_last < lo) return;
    const int hi = min(lo + kSegLen - 1, wave_last), kf = wave_last / kSegLen;
    GSTEX_STAT(0, 1);
    const float Af = 1.0f - T;
    float R = (Gimg[0] * bg0 + Gimg[1] * bg1) + Gimg[2] * bg2;
    float Gtex_bias = 0.f;  // tex_bias * sum_c dL/dtex[c]: the bias part of sum_c dL/dtex[c] * texel value
#pragma unroll
    for (int c = 0; c < CM; ++c) Gtex_bias += Gtex[c];
    Gtex_bias *= tex_bias;
    if (seg < kf) {
        // start from the forward's checkpoint after this segment: T_k, and R T_k = sum over the splats behind the
        // segment of w_j g_j + T_final (bg term) = (final - checkpoint accumulators) . upstream gradients
        const float* ck = aux.ckpt + ((size_t)slot * 4 + quad) * aux.F * 64 + lane;
        const float* fin = aux.ckpt + ((size_t)(sbase + kf) * 4 + quad) * aux.F * 64 + lane;
        const float Tk = ck[0];
        float back = (Gimg[0] * (fin[64] - ck[64]) + Gimg[1] * (fin[128] - ck[128])) + Gimg[2] * (fin[192] - ck[192]);
#pragma unroll
        for (int c = 0; c < CM; ++c)
            if (c < Cn) back += Gtex[c] * (fin[(4 + c) * 64] - ck[(4 + c) * 64]);
        back += Ga * (Tk - T);  // the weights behind sum to T_k - T_final
        if (GEO) {
            const float* fg = fin + (4 + Cn) * 64;
            const float* cg = ck + (4 + Cn) * 64;
            back += Gd * (fg[0] - cg[0]);
            back += (Gn[0] * (fg[64] - cg[64]) + Gn[1] * (fg[128] - cg[128])) + Gn[2] * (fg[192] - cg[192]);
            if (dreg) back += Greg * ((Af * (fg[320] - cg[320]) - 2.0f * M1f * (fg[256] - cg[256])) + M2f * (Tk - T));
        }
        if (inside) {
            R = (back + T * R) / Tk;
            T = Tk;
        }
    }
    float gabs = 0.f;  // max_c |dL/dtex[c]|: bounds this pixel's texel-gradient contributions (x w |tex_scale|)
#pragma unroll
    for (int c = 0; c < CM; ++c) gabs = fmaxf(gabs, fabsf(Gtex[c]));
    for (int i = lane; i < kTexStage; i += 64) s_texq[i] = 0;
    const size_t vm_base = visit_mask_base(rng.x, tile);

    for (int wd = hi >> 6; wd >= (lo >> 6); --wd) {
        const int pos0 = wd << 6;
        // the word's splats this wave visits: the forward's cull bits for this quadrant, clipped to the segment's
        // end (the wave's last contributor in the last segment)
        unsigned long long todo = aux.masks[(vm_base + wd) * 4 + quad];
        const int lim = hi - pos0 + 1;
        if (lim < 64) todo &= (1ull << lim) - 1ull;
        if (!todo) continue;
        // lane k <-> position pos0 + k: splat id and emission slot, loaded once per word (coalesced)
        int my_gid = 0, my_slot = 0;
        if ((todo >> lane) & 1ull) {
            my_gid = sorted_ids[rng.x + pos0 + lane];
            my_slot = sorted_slots[rng.x + pos0 + lane];
        }
#if GSTEX_WORD_WAIT
        // wait for the word's ids here, once: otherwise the waitcnt pass, which merges the loop's entry (ids
        // pending) with its back edge (the previous visit's atomics pending), waits at the top of EVERY visit for
        // all but one of the previous visit's atomics before the record can be addressed (vmcnt counts the
        // no-return atomics in order with the loads)
        asm volatile("; word ids %0 %1" ::"v"(my_gid), "v"(my_slot));
#endif
        while (todo) {
            const int j = 63 - __builtin_clzll(todo);
            todo &= ~(1ull << j);
            const int rel = pos0 + j;
            const int gid = __builtin_amdgcn_readlane(my_gid, j);
            const float4* rp = records + (size_t)gid * kRecF4;
            const Rec r = read_rec_global(rp);
            // one predicate for the whole heavy path (a single exec-mask region)
            Hit h;
            hit_p(r, px, py, h);
            // a near-edge-on splat (the record opacity's sign bit): p from its fp64 row, as in the forward
            if (hp_records && __float_as_int(rp[2].w) < 0) hit_p_hp(hp_records + (size_t)gid * H_FIELDS, px, py, h);
            const bool contrib = eval_rest(r, px, py, aa, h) && rel <= last;
            GSTEX_STAT(1, 1);
            GSTEX_STAT(3, __popcll(__ballot(contrib)));
            GSTEX_STAT(13, __popcll(__ballot(rel <= last)));           // lanes not yet past their last contributor
            GSTEX_STAT(14, __popcll(__ballot(contrib)) <= 16 ? 1 : 0);  // sparse visits
            GSTEX_STAT(15, __popcll(__ballot(contrib)) >= 48 ? 1 : 0);  // dense visits
            constexpr int NP = GEO ? kPartRowGeo : kPartRow;
            // a spare slot of the row (zero when stored): the texel fixed-point bound
            constexpr int kMBound = GEO ? 27 : P_NRM;
            float P[NP];
#pragma unroll
            for (int i = 0; i < NP; i += 2) {
                // zero rows in 64-bit moves (one v_mov_b64 per register pair)
                unsigned long long zz;
                asm volatile("v_mov_b64 %0, 0" : "=v"(zz));
                P[i] = __uint_as_float((unsigned)zz);
                P[i + 1] = __uint_as_float((unsigned)(zz >> 32));
            }
            // texel-gradient inputs, expanded into the 4*C bilinear contributions after P is reduced:
            // tkey = top-left texel of the block | (i1 - i0) << 29 | (j1 - j0) << 30, -1 if none
            int tkey = -1;
            float tw = 0.f, tax = 0.f, tay = 0.f;
            const bool blk_ok = r.off + r.h * r.w <= n_texels;  // wave-uniform; false only for corrupt dims
            if (contrib) {
                // gradient arithmetic only from here on (the pair decisions above are the forward's): contracted
#pragma clang fp contract(fast)
                const float one_m = 1.0f - h.alpha;
                T = T * grad_rcp(one_m);
                const float w = h.alpha * T;
                // issue the texel gathers first, then everything that does not need them
                const bool has_tex = r.h * r.w > 0 && blk_ok;
                Bilerp b;
                const __amdgpu_buffer_rsrc_t rs = texel_rsrc(texture, r.off, r.h * r.w, Cn);
                float t00[CM], t01[CM], t10[CM], t11[CM];
#pragma unroll
                for (int c = 0; c < CM; ++c) t00[c] = t01[c] = t10[c] = t11[c] = 0.f;
                if (has_tex) {
                    float xr, yr;
                    tex_coords(r, h.u, h.v, xr, yr);
                    // (converting h, w here measured faster than reading r.hf, r.wf)
                    b = bilerp_xy(xr, yr, r.h, r.w, (float)r.h - 1.0f, (float)r.w - 1.0f);
                    // (far corners unclamped: at a clamped edge their weight is 0 in the value and the edge's
                    // in_u / in_v = false drops the coordinate gradient, so the results are bit-identical)
                    if constexpr (CM == 3) {
                        load_texel_quad_unclamped(rs, b, r.w, t00, t01, t10, t11);
                    } else {
                        load_texel_quad<CM>(rs, b, r.w, Cn, t00, t01, t10, t11);
                    }
                }
                float g = (Gimg[0] * r.rgb[0] + Gimg[1] * r.rgb[1]) + Gimg[2] * r.rgb[2];
                P[P_RGB + 0] = w * Gimg[0];
                P[P_RGB + 1] = w * Gimg[1];
                P[P_RGB + 2] = w * Gimg[2];
                // depth: direct + distortion (m depends on z)
                float dz = 0.f, E = 0.f;
                if (GEO) {
                    P[P_NRM + 0] = w * Gn[0];
                    P[P_NRM + 1] = w * Gn[1];
                    P[P_NRM + 2] = w * Gn[2];
                    const float iz = grad_rcp(h.z);
                    const float m = kFarRatio * (1.0f - kNear * iz);
                    E = dreg ? ((m * m * Af - 2.0f * m * M1f) + M2f) : 0.0f;
                    dz = w * Gd;
                    if (dreg) dz += Greg * (2.0f * w * (m * Af - M1f)) * ((kFarRatio * kNear) * (iz * iz));
                }
                if (has_tex) {
                    tkey = (int)(__umul24(b.i0, r.w) + b.j0) | ((b.i1 - b.i0) << 29) | ((b.j1 - b.j0) << 30);
                    tw = w * tex_scale;  // d value / d stored texel
                    P[kMBound] = fabsf(tw) * gabs;  // summed by the reduce: the visit's fixed-point bound
                    tax = b.ax;
                    tay = b.ay;
                }
                // texture value (tex_scale * stored + tex_bias) and its uv-gradient.  Both are linear in the
                // texels, so the channels are folded first: D_k = sum_c Gtex[c] * t_k[c] per bilinear corner,
                // then one bilinear mix and one pair of differences serve all channels
                float dtu = 0.f, dtv = 0.f, dxr = 0.f, dyr = 0.f;
                if (has_tex) {
                    const float hf = (float)r.h, wf = (float)r.w;
                    float D00 = 0.f, D01 = 0.f, D10 = 0.f, D11 = 0.f;
#pragma unroll
                    for (int c = 0; c < CM; ++c) {
                        if (c < Cn) {
                            D00 = D00 + Gtex[c] * t00[c];
                            D01 = D01 + Gtex[c] * t01[c];
                            D10 = D10 + Gtex[c] * t10[c];
                            D11 = D11 + Gtex[c] * t11[c];
                        }
                    }
                    g += bilerp_mix(D00, D01, D10, D11, b.ax, b.ay) * tex_scale + Gtex_bias;
                    const float su = (1.0f - b.ay) * (D10 - D00) + b.ay * (D11 - D01);
                    const float sv = (1.0f - b.ax) * (D01 - D00) + b.ax * (D11 - D10);
                    // d value / d xr, d yr (texel units); the record's texture affine is prescaled by h, w
                    dxr = b.in_u ? w * su : 0.0f;
                    dyr = b.in_v ? w * sv : 0.0f;
                    dtu = dxr * hf;
                    dtv = dyr * wf;
                }
                if (GEO) {
                    g += Gd * h.z;
                    g += (Gn[0] * r.nrm[0] + Gn[1] * r.nrm[1]) + Gn[2] * r.nrm[2];
                }
                g += Ga;
                if (GEO) g += Greg * E;
                const float dL_dalpha = T * (g - R);
                R = h.alpha * g + one_m * R;

                float drho = 0.f;
                if (h.a_raw < kAlphaMax) {
                    P[P_OPAC] = dL_dalpha * h.G;
                    drho = dL_dalpha * h.a_raw * -0.5f;
                }
                GSTEX_PAIR(__int_as_float(gid), px, py, __int_as_float((h.use3 ? 1 : 0) | (h.a_raw < kAlphaMax ? 0 : 2)), T,
                           w, dL_dalpha, drho, h.u, h.v, h.ipz, h.z, h.alpha, h.G, h.dx, h.dy);
                // texture coordinates
                dtu *= tex_scale;  // the raw-value differences above, in value units
                dtv *= tex_scale;
                dxr *= tex_scale;
                dyr *= tex_scale;
                // gradients of the unscaled affine (uv0, auu, ...: what setup_bwd chains), and of u, v through the
                // prescaled one
                P[P_TU0] = dtu; P[P_AUU] = dtu * h.u; P[P_AUV] = dtu * h.v;
                P[P_TV0] = dtv; P[P_AVU] = dtv * h.u; P[P_AVV] = dtv * h.v;
                float du = dxr * r.auu + dyr * r.avu;
                float dv = dxr * r.auv + dyr * r.avv;
                // ray-splat (use3) vs screen-space low-pass branch, per lane, as selects
                const float du3 = GEO ? drho * 2.0f * h.u + dz * r.Tw.x : drho * 2.0f * h.u;
                const float dv3 = GEO ? drho * 2.0f * h.v + dz * r.Tw.y : drho * 2.0f * h.v;
                du = h.use3 ? du + du3 : du;
                dv = h.use3 ? dv + dv3 : dv;
                P[P_XY + 0] = h.use3 ? 0.f : drho * (2.0f * kFilterInvSq) * (r.x - px);
                P[P_XY + 1] = h.use3 ? 0.f : drho * (2.0f * kFilterInvSq) * (r.y - py);
                const float ipz = h.ipz;
                const f3 dp = f3{du * ipz, dv * ipz, -(du * h.u + dv * h.v) * ipz};
                // p = dx A + dy B + P0 (affine form): dL/dA = dp dx, dL/dB = dp dy, dL/dP0 = dp
                P[P_A + 0] = dp.x * h.dx; P[P_A + 1] = dp.y * h.dx; P[P_A + 2] = dp.z * h.dx;
                P[P_B + 0] = dp.x * h.dy; P[P_B + 1] = dp.y * h.dy; P[P_B + 2] = dp.z * h.dy;
                P[P_P0 + 0] = dp.x; P[P_P0 + 1] = dp.y; P[P_P0 + 2] = dp.z;
                if constexpr (GEO) {  // the depth's direct dependence on Tw (z = u Tw.x + v Tw.y + Tw.z)
                    P[P_TW + 0] = h.use3 ? dz * h.u : 0.f;
                    P[P_TW + 1] = h.use3 ? dz * h.v : 0.f;
                    P[P_TW + 2] = dz;
                }
            }
            float vis_M = 0.f;  // sum over the wave's pixels of |w tex_scale| max_c |dL/dtex[c]| for this splat
            if (__any(contrib)) {
                GSTEX_STAT(2, 1);
                wave_reduce<NP>(P);
                // take the bound out of the spare slot (kMBound) before the row is stored
                constexpr int kML = GEO ? 48 : 56, kMI = GEO ? 3 : 0;  // its lane and index after the reduce-scatter
                vis_M = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(P[kMI]), kML));
                if (lane == kML) P[kMI] = 0.0f;
                // lanes 8k hold NP / 8 consecutive values each.  Deterministic mode (row_flags given): the
                // (pair, quadrant) row, whose flag (1: 24-value row, 2: 32-value row) marks it written, summed by
                // setup_bwd in a fixed order.  Otherwise: added with float atomics into the splat's NP-value
                // accumulator row (zeroed by the caller): no row traffic, no summing pass, order-dependent rounding
                constexpr int E = NP / 8;
                const int base = (NP / 2) * ((lane >> 5) & 1) + (NP / 4) * ((lane >> 4) & 1) + E * ((lane >> 3) & 1);
                if (row_flags) {
                    const int slot = __builtin_amdgcn_readlane(my_slot, j);
                    if ((lane & 7) == 0) {
                        float* dst = partials + ((size_t)slot * 4 + quad) * NP + base;  // rows NP floats apart
                        if constexpr (E == 4) {
                            *reinterpret_cast<float4*>(dst) = make_float4(P[0], P[1], P[2], P[3]);
                        } else {
                            dst[0] = P[0];
                            dst[1] = P[1];
                            dst[2] = P[2];
                        }
                    }
                    if (lane == 0) row_flags[(size_t)slot * 4 + quad] = GEO ? 2 : 1;
                } else {
                    float* dst = partials + (size_t)gid * NP + base;
                    // lane 8k + e takes value e of lane 8k (DPP row shifts): one atomic instruction covers the NP
                    // contiguous floats (2 cache-line requests; E atomics from each lane 8k measured +0.2 ms)
                    const int e = lane & 7;
                    float v = P[0];
                    const float s1 = dpp_shr_f<1>(P[1]), s2 = dpp_shr_f<2>(P[2]);
                    v = e == 1 ? s1 : v;
                    v = e == 2 ? s2 : v;
                    if constexpr (E == 4) {
                        const float s3 = dpp_shr_f<3>(P[3]);
                        v = e == 3 ? s3 : v;
                    }
                    if (e < E) atomicAdd(dst + e, v);
                }
            }
            if (__any(tkey >= 0)) {
                // fixed point for this visit: every staged entry receives at most vis_M in value units (bilinear
                // weights <= 1), so at scale 2^S, S = 30 - e (vis_M < 2^e), the tails (each < 2^30) and their int32
                // sums stay in range; resolution 2^-30 of the visit's total
                // S = 30 - e with vis_M = m 2^e, m in [0.5, 1) (frexp), from the float's exponent field on the scalar
                // unit (vis_M is wave-uniform); 2^S and 2^-S are built as float bit patterns, so the scalings below
                // are exact multiplies (what ldexp computed); S is clamped to [-126, 126] (denormal / zero bounds)
                const uint32_t mbits = (uint32_t)__builtin_amdgcn_readfirstlane((int)__float_as_uint(vis_M));
                const int biased = (int)((mbits >> 23) & 0xFFu);
                const int e_m = biased > 0 ? biased - 126 : 0;
                const int tex_S = min(max(kTexFixBits - e_m, -126), 126);
                const float pow_S = __uint_as_float((uint32_t)(tex_S + 127) << 23);     // 2^S
                const float pow_mS = __uint_as_float((uint32_t)(127 - tex_S) << 23);    // 2^-S
                const float twq = tw * pow_S;
                float tg[4 * CM];
                {
#pragma clang fp contract(fast)
                    const float fi0 = 1.0f - tax, fi1 = tax, fj0 = 1.0f - tay, fj1 = tay;
                    const float w00 = fi0 * fj0, w01 = fi0 * fj1;
                    const float w10 = fi1 * fj0, w11 = fi1 * fj1;
#pragma unroll
                    for (int c = 0; c < CM; ++c) {
                        const float gt = (c < Cn) ? twq * Gtex[c] : 0.0f;
                        tg[c] = gt * w00;
                        tg[CM + c] = gt * w01;
                        tg[2 * CM + c] = gt * w10;
                        tg[3 * CM + c] = gt * w11;
                    }
                }
                const bool tail = seg_reduce_rows<4 * CM>(tkey, tg);
                const int bsize = r.h * r.w * Cn;  // wave-uniform
                const bool staged = bsize <= kTexStage;
                GSTEX_STAT(5, __popcll(__ballot(tail)));
                GSTEX_STAT(7, 1);
                if (tail) {
                    const int t0 = tkey & ((1 << 29) - 1), tdi = (tkey >> 29) & 1, tdj = (tkey >> 30) & 1;
                    const int c00 = t0 * Cn, c01 = (t0 + tdj) * Cn;
                    const int c10 = (t0 + tdi * r.w) * Cn, c11 = (t0 + tdi * r.w + tdj) * Cn;
                    if (staged) {
#pragma unroll
                        for (int c = 0; c < CM; ++c) {
                            if (c < Cn) {
                                stage_add(&s_texq[c00 + c], tg[c]);
                                stage_add(&s_texq[c01 + c], tg[CM + c]);
                                stage_add(&s_texq[c10 + c], tg[2 * CM + c]);
                                stage_add(&s_texq[c11 + c], tg[3 * CM + c]);
                            }
                        }
                    } else {
                        // block larger than the staging area: straight to global, back in value units
                        float* base = v_texture + (size_t)r.off * Cn;
                        auto val = [&](float y) { return y * pow_mS; };
#pragma unroll
                        for (int c = 0; c < CM; ++c) {
                            if (c < Cn) {
                                atomicAdd(base + c00 + c, val(tg[c]));
                                atomicAdd(base + c01 + c, val(tg[CM + c]));
                                atomicAdd(base + c10 + c, val(tg[2 * CM + c]));
                                atomicAdd(base + c11 + c, val(tg[3 * CM + c]));
                            }
                        }
                    }
                }
                if (staged) {
                    // flush the block (non-zero entries only) and leave the staging area zeroed; the wave's LDS
                    // operations complete in order, so these reads see every tail added above
                    float* dst = v_texture + (size_t)r.off * Cn;
                    // kFlushU entries per lane per pass, their LDS reads issued together (one wait per pass); entries
                    // past the block are zero (the staging area is kept zeroed) and kTexStage is a multiple of the pass
                    for (int e0 = lane; e0 < bsize; e0 += 64 * kFlushU) {
                        int v[kFlushU];
                        GSTEX_STAT(4, 1);
#pragma unroll
                        for (int k = 0; k < kFlushU; ++k) v[k] = s_texq[e0 + 64 * k];
#pragma unroll
                        for (int k = 0; k < kFlushU; ++k) {
                            GSTEX_STAT(6, __popcll(__ballot(v[k] != 0)));
                            if (v[k] == 0) continue;
                            s_texq[e0 + 64 * k] = 0;
                            atomicAdd(dst + e0 + 64 * k, (float)v[k] * pow_mS);
                        }
                    }
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// setup backward: sum partials per splat, chain to parameters
// ------------------------------------------------------------------------------------------
constexpr int kSetupBwdRows = 8;  // splats summed per 256-thread workgroup (32 lanes each)
#ifndef GSTEX_SUM_SLOTS
#define GSTEX_SUM_SLOTS 8
#endif
constexpr int kSumSlots = GSTEX_SUM_SLOTS;  // slots whose rows one lane group has in flight at once (16: equal; 4: slower)
// Deterministic mode: setup_bwd_sum_kernel, 32 lanes per splat, sums the splat's flagged rows in (slot, quadrant)
// order and writes the 32 sums over the splat's first row (slot offsets[g], quadrant 0), whose values it has already
// read -- no other splat reads that row; then setup_bwd_chain_kernel, one thread per splat, chains the sums to the
// parameters.  (One fused kernel, 40 splats per workgroup, measured 120 vs 102 us in round 2.)
// Capacity mode (n_rows >= 0, gstex_bin_sort_capped): a total offsets[n] above the row capacity means the binning
// left every tile empty and no row was written; both kernels then treat every splat as pair-free (zero gradients)
// instead of addressing rows past the buffers.
// 32 lanes per splat: lane 8 q + m reads float4 m (columns 4m .. 4m+3) of the quadrant-q rows, kSumSlots slots at a
// time, and sums them in slot order; the 4 quadrant sums are then combined (q0 + q1) + (q2 + q3) across lanes.
// Deterministic (fixed order), like the fused kernel's slot-major quadrant-minor order it replaces.
// rs = floats between rows: kPartRow (24) when the backward had no depth / normal / distortion gradient, else
// kPartRowGeo (32).  The sums (32 values, the last 8 zero for 24-value rows) go over the splat's first row; with rs =
// 24 they reach into its second row, which only this splat's lanes read, before (program order) the store.
__global__ __launch_bounds__(256) void setup_bwd_sum_kernel(int n, const int32_t* __restrict__ nth,
                                                           const int32_t* __restrict__ offsets,
                                                           float* __restrict__ partials,
                                                           const uint32_t* __restrict__ row_flags, int rs,
                                                           int64_t n_rows) {
    const int l = threadIdx.x & 31, q = l >> 3, m = l & 7;
    const int g = blockIdx.x * 8 + (threadIdx.x >> 5);
    const bool live = g < n && !(n_rows >= 0 && (int64_t)offsets[n] > n_rows);  // over capacity: no rows exist
    const int cnt = live ? nth[g] : 0;
    const size_t s0 = live ? (size_t)offsets[g] : 0;
    // columns 24.. exist only in 32-value rows (flag 2: backward with depth / normal gradients)
    const uint32_t need = m < kPartRow / 4 ? 0xFFu : 0x02u;
    const float4* rows = reinterpret_cast<const float4*>(partials + s0 * 4 * rs) + q * (rs / 4) + m;
    const uint32_t* fl = row_flags + s0;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int e = 0; e < cnt; e += kSumSlots) {
        uint32_t f[kSumSlots];
#pragma unroll
        for (int u = 0; u < kSumSlots; ++u) f[u] = e + u < cnt ? fl[e + u] : 0u;
        float4 r[kSumSlots];
#pragma unroll
        for (int u = 0; u < kSumSlots; ++u)
            r[u] = (f[u] >> (8 * q)) & need ? rows[(size_t)(e + u) * rs] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < kSumSlots; ++u) {
            if ((f[u] >> (8 * q)) & need) {
                acc.x += r[u].x;
                acc.y += r[u].y;
                acc.z += r[u].z;
                acc.w += r[u].w;
            }
        }
    }
    // (q0 + q1) + (q2 + q3): lane l adds lane l ^ 8, then lane l ^ 16 (inside the 32-lane splat group)
    auto xadd = [](float4 a, int mask) {
        return make_float4(a.x + __shfl_xor(a.x, mask, 32), a.y + __shfl_xor(a.y, mask, 32),
                           a.z + __shfl_xor(a.z, mask, 32), a.w + __shfl_xor(a.w, mask, 32));
    };
    acc = xadd(acc, 8);
    acc = xadd(acc, 16);
    // the sums over the splat's first row, whose values every lane has read above: no other splat reads it
    if (live && cnt > 0 && q == 0)
        reinterpret_cast<float4*>(partials + s0 * 4 * rs)[m] = acc;
}

template <bool FOLD_AABB>
__device__ __forceinline__ void setup_bwd_chain(int g, const float (&S)[kPartRowGeo], int cnt, const Camera& cam,
    const float* __restrict__ means, const float* __restrict__ scales, float glob,
    const float* __restrict__ quats, const float* __restrict__ umap, const float* __restrict__ vmap,
    float* __restrict__ v_means, float* __restrict__ v_scales, float* __restrict__ v_quats,
    float* __restrict__ v_rgbs, float* __restrict__ v_opac, float* __restrict__ v_centers, float* __restrict__ v_uv0);

template <bool FOLD_AABB>
__global__ __launch_bounds__(256) void setup_bwd_chain_kernel(
    int n, const float* __restrict__ means, const float* __restrict__ scales, float glob,
    const float* __restrict__ quats, const float* __restrict__ umap, const float* __restrict__ vmap,
    const int32_t* __restrict__ nth, const int32_t* __restrict__ offsets, const float* __restrict__ partials, int rs,
    bool per_splat, int64_t n_rows, CamArgs cam_args, float* __restrict__ v_means, float* __restrict__ v_scales,
    float* __restrict__ v_quats, float* __restrict__ v_rgbs, float* __restrict__ v_opac, float* __restrict__ v_centers,
    float* __restrict__ v_uv0) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= n) return;
    const Camera cam = load_camera(cam_args);
    // deterministic mode over capacity (n_rows >= 0): the binning left every tile empty and no row exists
    const bool over = !per_splat && n_rows >= 0 && (int64_t)offsets[n] > n_rows;
    const int cnt = over ? 0 : nth[g];
    float S[kPartRowGeo];
    if (per_splat) {
        // the backward's (N, rs) accumulator rows (zero for a splat without pairs): all eight 16-B loads issued at
        // once, in bounds (a 24-value row re-reads its last vector), independent of the pair count's load
        const float4* src = reinterpret_cast<const float4*>(partials + (size_t)g * rs);
        const int n4 = rs / 4;
#pragma unroll
        for (int i = 0; i < kPartRowGeo / 4; ++i) {
            const float4 v = src[i < n4 ? i : n4 - 1];
            const bool use = i < n4 && cnt > 0;
            S[4 * i] = use ? v.x : 0.f; S[4 * i + 1] = use ? v.y : 0.f;
            S[4 * i + 2] = use ? v.z : 0.f; S[4 * i + 3] = use ? v.w : 0.f;
        }
    } else if (cnt > 0) {
        // the sums setup_bwd_sum wrote over the splat's first partial row (32 values, the last 8 zero for 24-value
        // rows)
        const float4* src = reinterpret_cast<const float4*>(partials + (size_t)offsets[g] * 4 * rs);
#pragma unroll
        for (int i = 0; i < kPartRowGeo / 4; ++i) {
            const float4 v = src[i];
            S[4 * i] = v.x; S[4 * i + 1] = v.y; S[4 * i + 2] = v.z; S[4 * i + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kPartRowGeo; ++i) S[i] = 0.f;
    }
    setup_bwd_chain<FOLD_AABB>(g, S, cnt, cam, means, scales, glob, quats, umap, vmap, v_means, v_scales, v_quats,
                               v_rgbs, v_opac, v_centers, v_uv0);
}

template <bool FOLD_AABB>
__device__ __forceinline__ void setup_bwd_chain(int g, const float (&S)[kPartRowGeo], int cnt, const Camera& cam,
    const float* __restrict__ means, const float* __restrict__ scales, float glob,
    const float* __restrict__ quats, const float* __restrict__ umap, const float* __restrict__ vmap,
    float* __restrict__ v_means, float* __restrict__ v_scales, float* __restrict__ v_quats,
    float* __restrict__ v_rgbs, float* __restrict__ v_opac, float* __restrict__ v_centers, float* __restrict__ v_uv0) {
    v_rgbs[3 * g + 0] = S[P_RGB + 0];
    v_rgbs[3 * g + 1] = S[P_RGB + 1];
    v_rgbs[3 * g + 2] = S[P_RGB + 2];
    v_opac[g] = S[P_OPAC];
    v_centers[2 * g + 0] = S[P_XY + 0];
    v_centers[2 * g + 1] = S[P_XY + 1];
    v_uv0[2 * g + 0] = S[P_TU0];
    v_uv0[2 * g + 1] = S[P_TV0];
    if (cnt <= 0) {
        v_means[3 * g] = v_means[3 * g + 1] = v_means[3 * g + 2] = 0.f;
        v_scales[3 * g] = v_scales[3 * g + 1] = v_scales[3 * g + 2] = 0.f;
        v_quats[4 * g] = v_quats[4 * g + 1] = v_quats[4 * g + 2] = v_quats[4 * g + 3] = 0.f;
        return;
    }
    // fp64 chain (one thread per splat): the record it differentiates was evaluated in fp64 (setup_kernel)
    const FrameT<double> fr = quat_frame_t<double>(quats + 4 * g);
    const double su = (double)scales[3 * g] * (double)glob, sv = (double)scales[3 * g + 1] * (double)glob;
    const d3 mu = d3{(double)means[3 * g], (double)means[3 * g + 1], (double)means[3 * g + 2]};
    const AnchoredT<double> an = splat_anchored(cam, mu, su, sv, fr);
    d3 dTu, dTv, dTw;
    auto sd = [&](int i) { return d3{(double)S[i], (double)S[i + 1], (double)S[i + 2]}; };
    affine_homog_vjp(an.Tu, an.Tv, an.Tw, sd(P_A), sd(P_B), sd(P_P0), dTu, dTv, dTw);
    dTw = add3(dTw, sd(P_TW));
    const HomogGradT<double> hg = splat_anchored_vjp(cam, su, sv, fr, an.xn, an.yn, dTu, dTv, dTw);
    const d3 um = d3{(double)umap[3 * g], (double)umap[3 * g + 1], (double)umap[3 * g + 2]};
    const d3 vm = d3{(double)vmap[3 * g], (double)vmap[3 * g + 1], (double)vmap[3 * g + 2]};
    const double dauu = S[P_AUU], dauv = S[P_AUV], davu = S[P_AVU], davv = S[P_AVV];
    const double dsu = hg.dsu + dauu * dot3(fr.tu, um) + davu * dot3(fr.tu, vm);
    const double dsv = hg.dsv + dauv * dot3(fr.tv, um) + davv * dot3(fr.tv, vm);
    const d3 dtu = add3(hg.dtu, add3(scale3(um, dauu * su), scale3(vm, davu * su)));
    const d3 dtv = add3(hg.dtv, add3(scale3(um, dauv * sv), scale3(vm, davv * sv)));
    const d3 dir = d3{(double)cam.campos[0] - mu.x, (double)cam.campos[1] - mu.y, (double)cam.campos[2] - mu.z};
    const double sgn = dot3(fr.tw, dir) < 0.0 ? -1.0 : 1.0;
    const d3 dtw = d3{sgn * S[P_NRM], sgn * S[P_NRM + 1], sgn * S[P_NRM + 2]};
    double dqd[4];
    frame_vjp(fr, dtu, dtv, dtw, dqd);
    // rounded to fp32 once; the folded AABB-centre chain below stays fp32 (bit-identical to get_aabb_2d's backward)
    f3 vmu = to_f3(hg.dmu);
    float vsu = (float)(dsu * (double)glob), vsv = (float)(dsv * (double)glob);
    float dq[4] = {(float)dqd[0], (float)dqd[1], (float)dqd[2], (float)dqd[3]};
    if (FOLD_AABB) {
        // aabb_bwd_kernel for this splat (zero when there is no centre gradient or the splat is culled)
        f3 amu = f3{0.f, 0.f, 0.f};
        float asu = 0.f, asv = 0.f, aq[4] = {0.f, 0.f, 0.f, 0.f};
        const float gcx = S[P_XY + 0], gcy = S[P_XY + 1];
        float acx, acy, aex, aey;
        const Frame frf = quat_frame(quats + 4 * g);
        const float suf = scales[3 * g] * glob, svf = scales[3 * g + 1] * glob;
        const Homog ah = splat_homography(cam, mk3(means[3 * g], means[3 * g + 1], means[3 * g + 2]), suf, svf, frf);
        if (!(gcx == 0.0f && gcy == 0.0f) && aabb_from_homog(ah, acx, acy, aex, aey)) {
            f3 dTu, dTv, dTw;
            aabb_centre_vjp(ah, acx, acy, gcx, gcy, dTu, dTv, dTw);
            const HomogGrad ag = splat_homography_vjp(cam, suf, svf, frf, dTu, dTv, dTw);
            frame_vjp(frf, ag.dtu, ag.dtv, f3{0.0f, 0.0f, 0.0f}, aq);
            amu = ag.dmu;
            asu = ag.dsu * glob;
            asv = ag.dsv * glob;
        }
        vmu = add3(vmu, amu);
        vsu = vsu + asu;
        vsv = vsv + asv;
#pragma unroll
        for (int k = 0; k < 4; ++k) dq[k] = dq[k] + aq[k];
    }
    v_means[3 * g + 0] = vmu.x;
    v_means[3 * g + 1] = vmu.y;
    v_means[3 * g + 2] = vmu.z;
    v_scales[3 * g + 0] = vsu;
    v_scales[3 * g + 1] = vsv;
    v_scales[3 * g + 2] = 0.f;
    v_quats[4 * g + 0] = dq[0];
    v_quats[4 * g + 1] = dq[1];
    v_quats[4 * g + 2] = dq[2];
    v_quats[4 * g + 3] = dq[3];
}

// ------------------------------------------------------------------------------------------
// texture_edit (gstex.py:579-606, viewer paint tool): splat a screen-space RGBA stroke into the
// texel store.  Same front-to-back traversal as the forward (same cull, termination and weights
// w = alpha * T); a pair whose hit depth lies inside the pixel's [depth_lo, depth_hi] window (the
// caller passes the rendered depth +- 1e-2) adds, for each of its 4 bilinear texels with weight b,
//   out[texel] += b * w * (a * r, a * g, a * b, a, 1)
// so out[:, :3] / out[:, 3] is the stroke colour and out[:, 3] / out[:, 4] the blend weight the caller
// forms (gstex.py:602-605).  Viewer path: global float atomics, no LDS staging.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void texture_edit_kernel(
    CamArgs cam_args, int tiles_x, int settings, const float4* __restrict__ records,
    const int2* __restrict__ tile_ranges, const int32_t* __restrict__ tile_order, const int32_t* __restrict__ sorted_ids,
    const float* __restrict__ edit_rgb, const float* __restrict__ edit_a, const float* __restrict__ depth_lo,
    const float* __restrict__ depth_hi, int n_texels, float* __restrict__ out) {
    const Camera cam = load_camera(cam_args);
    __shared__ float4 s_rec[kRecF4 * kFwdBatch];
    const int tile = tile_order ? tile_order[blockIdx.x] : (int)blockIdx.x;
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    const int tid = threadIdx.x;
    const WaveBlock wb = wave_block(tx, ty, tid);
    const int pxi = wb.px, pyi = wb.py;
    const bool inside = pxi < cam.W && pyi < cam.H;
    const float px = (float)pxi + 0.5f, py = (float)pyi + 0.5f;  // pixel centres (gstex_common.h)
    const bool aa = (settings & GSTEX_SETTING_AA_BLUR) != 0;
    const int2 rng = tile_ranges[tile];
    float er = 0.f, eg = 0.f, eb = 0.f, ea = 0.f, dlo = 1.0f, dhi = 0.0f;
    if (inside) {
        const size_t pix = (size_t)pyi * cam.W + pxi;
        er = edit_rgb[3 * pix]; eg = edit_rgb[3 * pix + 1]; eb = edit_rgb[3 * pix + 2];
        ea = edit_a[pix];
        dlo = depth_lo[pix];
        dhi = depth_hi[pix];
    }
    float T = 1.0f;
    bool done = !inside;
    for (int b0 = rng.x; b0 < rng.y; b0 += kFwdBatch) {
        if (__syncthreads_count(done ? 1 : 0) == kThreads) break;
        for (int q = tid; q < kFwdBatch * kRecF4; q += kThreads) {
            const int j = q / kRecF4, k = q % kRecF4;
            if (b0 + j < rng.y) s_rec[k * kFwdBatch + j] = records[(size_t)sorted_ids[b0 + j] * kRecF4 + k];
        }
        __syncthreads();
        const int nb = min(kFwdBatch, rng.y - b0);
        for (int j = 0; j < nb && !done; ++j) {
            if (!wave_may_hit<kFwdBatch>(s_rec, j, wb.wx0, wb.wx1, wb.wy0, wb.wy1, aa)) continue;
            const Rec r = read_rec<kFwdBatch>(s_rec, j);
            Hit h;
            if (!eval_hit(r, px, py, aa, h)) continue;
            const float test_T = T * (1.0f - h.alpha);
            if (test_T < kTMin) {
                done = true;
                break;
            }
            const float w = h.alpha * T;
            if (r.h * r.w > 0 && r.off + r.h * r.w <= n_texels && h.z >= dlo && h.z <= dhi) {
                float tu, tv;
                tex_coords(r, h.u, h.v, tu, tv);
                const Bilerp bl = bilerp_xy(tu, tv, r.h, r.w, r.hm1, r.wm1);
                const float wc[4] = {(1.0f - bl.ax) * (1.0f - bl.ay), (1.0f - bl.ax) * bl.ay,
                                     bl.ax * (1.0f - bl.ay), bl.ax * bl.ay};
                const int tc[4] = {bl.i0 * r.w + bl.j0, bl.i0 * r.w + bl.j1, bl.i1 * r.w + bl.j0, bl.i1 * r.w + bl.j1};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float bw = wc[k] * w, baw = bw * ea;
                    float* o = out + (size_t)(r.off + tc[k]) * 5;
                    atomicAdd(o + 0, baw * er);
                    atomicAdd(o + 1, baw * eg);
                    atomicAdd(o + 2, baw * eb);
                    atomicAdd(o + 3, baw);
                    atomicAdd(o + 4, bw);
                }
            }
            T = test_T;
        }
        __syncthreads();
    }
}

int check_settings(int settings) {
    const int known = GSTEX_SETTING_AA_BLUR | GSTEX_SETTING_DIST_REG | GSTEX_SETTING_EVAL_NORMAL;
    if (settings & ~known) {
        set_error("texture_gaussians: unsupported settings bits 0x%x (supported: 1<<9, 1<<10, 1<<15)",
                  settings & ~known);
        return GSTEX_ERR_UNSUPPORTED;
    }
    return GSTEX_OK;
}

// The training render's backward after the raster backward, one thread per splat (gstex_train_epilogue, ABI 17): the
// record chain of setup_bwd_chain_kernel<true> (fast mode: the per-splat accumulator rows), then the activations'
// backward (activate_bwd_splat) and the SH rest coefficients' backward (sh_grad_row, the rows staged in LDS and copied
// out contiguously) on the chain's outputs -- the functions gstex_raster_setup_bwd_aabb, gstex_activate_bwd and
// gstex_sh_rest_bwd run, on the same values: bit-identical gradients, two launches fewer.
constexpr int kEpiBlock = 256;
__global__ __launch_bounds__(kEpiBlock) void train_epilogue_kernel(
    int n, int degree, int n_rest, CamArgs cam_args, const float* __restrict__ means, const float* __restrict__ scales,
    const float* __restrict__ quats_n, const float* __restrict__ quats, const float* __restrict__ log_scales,
    const float* __restrict__ opacities, const float* __restrict__ umap, const float* __restrict__ vmap,
    const float* __restrict__ viewdirs, const int32_t* __restrict__ nth, const float* __restrict__ partials,
    float* __restrict__ v_means, float* __restrict__ v_quats, float* __restrict__ v_log_scales,
    float* __restrict__ v_opac_logits, float* __restrict__ v_rest, float* __restrict__ v_scales_act,
    float* __restrict__ v_quats_n, float* __restrict__ v_rgbs, float* __restrict__ v_opac_act,
    float* __restrict__ v_centers, float* __restrict__ v_uv0) {
    extern __shared__ float s_row[];
    const int t = threadIdx.x;
    const int i0 = blockIdx.x * kEpiBlock;
    const int cnt_blk = min(kEpiBlock, n - i0);
    const int kw = n_rest * 3;
    if (t < cnt_blk) {
        const int g = i0 + t;
        const Camera cam = load_camera(cam_args);
        const int cnt = nth[g];
        float S[kPartRowGeo];
        const float4* src = reinterpret_cast<const float4*>(partials + (size_t)g * kPartRow);
        constexpr int n4 = kPartRow / 4;
#pragma unroll
        for (int i = 0; i < kPartRowGeo / 4; ++i) {
            const float4 v = src[i < n4 ? i : n4 - 1];
            const bool use = i < n4 && cnt > 0;
            S[4 * i] = use ? v.x : 0.f; S[4 * i + 1] = use ? v.y : 0.f;
            S[4 * i + 2] = use ? v.z : 0.f; S[4 * i + 3] = use ? v.w : 0.f;
        }
        setup_bwd_chain<true>(g, S, cnt, cam, means, scales, 1.0f, quats_n, umap, vmap, v_means, v_scales_act,
                              v_quats_n, v_rgbs, v_opac_act, v_centers, v_uv0);
        // (this thread's own stores, read back)
        float4 vq;
        float vls0, vls1, vo;
        activate_bwd_splat(reinterpret_cast<const float4*>(quats)[g], log_scales[3 * g], log_scales[3 * g + 1],
                           opacities[g], reinterpret_cast<const float4*>(v_quats_n)[g], v_scales_act[3 * g],
                           v_scales_act[3 * g + 1], v_opac_act[g], vq, vls0, vls1, vo);
        reinterpret_cast<float4*>(v_quats)[g] = vq;
        v_log_scales[3 * g] = vls0;
        v_log_scales[3 * g + 1] = vls1;
        v_log_scales[3 * g + 2] = 0.0f;
        v_opac_logits[g] = vo;
        sh_grad_row(degree, 1, n_rest, viewdirs[3 * g], viewdirs[3 * g + 1], viewdirs[3 * g + 2], v_rgbs[3 * g],
                    v_rgbs[3 * g + 1], v_rgbs[3 * g + 2], s_row + t * kw);
    }
    __syncthreads();
    sh_copy_span<kEpiBlock>(v_rest + (size_t)i0 * kw, s_row, cnt_blk * kw);
}

}  // namespace

namespace gstex {
ZeroSpan raster_aux_zero_span(void* aux, int64_t n_isect, int32_t n_tiles, int32_t channels) {
    const AuxLayout al = aux_layout(n_isect, n_tiles, channels);
    return ZeroSpan{aux ? (char*)aux + al.cost : nullptr, al.order_ws - al.cost + (size_t)2 * kUnitBins * 4};
}
}  // namespace gstex

extern "C" int gstex_raster_setup(int32_t n, const float* means, const float* scales, float glob_scale,
                                  const float* quats, const float* rgbs, const float* opacities,
                                  const float* centers, const float* uv0, const float* umap, const float* vmap,
                                  const int32_t* texture_dims, const int32_t* num_tiles_hit,
                                  const gstex_camera* cam, float* records, double* hp_records, void* stream) {
    GSTEX_REQUIRE(n >= 0 && cam, "gstex_raster_setup: invalid arguments");
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(means && scales && quats && rgbs && opacities && centers && uv0 && umap && vmap &&
                      texture_dims && num_tiles_hit && records,
                  "gstex_raster_setup: null pointer");
    setup_kernel<<<div_up(n, 256), 256, 0, as_stream(stream)>>>(n, means, scales, glob_scale, quats, rgbs, opacities,
                                                                 centers, uv0, umap, vmap, texture_dims,
                                                                 num_tiles_hit, to_device_camera(*cam), records,
                                                                 hp_records);
    return launch_status("gstex_raster_setup");
}

extern "C" int gstex_raster_fwd(const gstex_camera* cam, int32_t channels, int32_t settings,
                                const float* background, const float* records, const double* hp_records,
                                const int32_t* tile_ranges,
                                const int32_t* tile_order, const int32_t* sorted_ids, const float* texture,
                                int64_t n_texels, float tex_scale, float tex_bias, float* out_img, float* out_depth, float* out_reg, float* out_alpha, float* out_tex,
                                float* out_normal, float* state, int64_t n_isect, void* aux, void* stream) {
    return gstex_raster_fwd_zero(cam, channels, settings, background, records, hp_records, tile_ranges, tile_order,
                                 sorted_ids,
                                 texture, n_texels, tex_scale, tex_bias, out_img, out_depth, out_reg, out_alpha,
                                 out_tex, out_normal, state, n_isect, aux, nullptr, 0, nullptr, 0, stream);
}

extern "C" int gstex_raster_fwd_zero(const gstex_camera* cam, int32_t channels, int32_t settings,
                                     const float* background, const float* records, const double* hp_records,
                                     const int32_t* tile_ranges,
                                     const int32_t* tile_order, const int32_t* sorted_ids, const float* texture,
                                     int64_t n_texels, float tex_scale, float tex_bias, float* out_img,
                                     float* out_depth, float* out_reg, float* out_alpha, float* out_tex,
                                     float* out_normal, float* state, int64_t n_isect, void* aux, float* zero_buf,
                                     int64_t zero_floats, float* zero_buf2, int64_t zero_floats2, void* stream) {
    GSTEX_REQUIRE(zero_floats >= 0 && (zero_floats == 0 || zero_buf) && zero_floats2 >= 0 &&
                  (zero_floats2 == 0 || zero_buf2), "gstex_raster_fwd: invalid zero_buf / zero_floats");
    GSTEX_REQUIRE(cam && cam->H > 0 && cam->W > 0, "gstex_raster_fwd: invalid camera");
    GSTEX_REQUIRE(cam->block == kTile, "gstex_raster_fwd: block_width must be %d (got %d)", kTile, cam->block);
    GSTEX_REQUIRE(channels >= 1 && channels <= 8, "gstex_raster_fwd: channels must be in [1, 8] (got %d)",
                  channels);
    GSTEX_REQUIRE(n_texels >= 0 && n_texels * channels < (int64_t)INT32_MAX, "gstex_raster_fwd: n_texels out of range");
    GSTEX_REQUIRE(n_texels == 0 || texture, "gstex_raster_fwd: null texture");
    int rc = check_settings(settings & ~GSTEX_SETTING_AUX_ZEROED);
    if (rc) return rc;
    GSTEX_REQUIRE(tile_ranges && out_img && out_alpha && out_tex && state, "gstex_raster_fwd: null pointer");
    const bool geo = out_depth || out_reg || out_normal;
    GSTEX_REQUIRE(!geo || (out_depth && out_reg && out_normal),
                  "gstex_raster_fwd: out_depth, out_reg and out_normal must be all given or all NULL");
    GSTEX_REQUIRE(n_isect >= 0 && n_isect < (int64_t)INT32_MAX, "gstex_raster_fwd: n_isect out of range");
    const int tiles_x = (cam->W + kTile - 1) / kTile, tiles_y = (cam->H + kTile - 1) / kTile;
    CamArgs dc = to_device_camera(*cam);
    hipStream_t st = as_stream(stream);
    const int nblk = tiles_x * tiles_y;
    const AuxLayout al = aux_layout(n_isect, nblk, channels);
    const AuxPtrs ap = aux_ptrs(aux, al);
    // one fill: unit costs (units the forward never reaches keep 0; the backward skips them), the launch order
    // (0 = no unit at that position) and the unit-order histogram the forward builds (contiguous in the layout)
    if (aux && !(settings & GSTEX_SETTING_AUX_ZEROED) &&
        hipMemsetAsync(ap.cost, 0, al.order_ws - al.cost + (size_t)2 * kUnitBins * 4, st) != hipSuccess)
        return launch_status("gstex_raster_fwd (aux)");
    settings &= ~GSTEX_SETTING_AUX_ZEROED;
    ZeroBufs zbuf;
    zbuf.p[0] = zero_floats > 0 ? zero_buf : nullptr;
    zbuf.n[0] = zero_floats;
    zbuf.p[1] = zero_floats2 > 0 ? zero_buf2 : nullptr;
    zbuf.n[1] = zero_floats2;
    int fgrid = fwd_grid(tiles_x, tiles_y);
#define GSTEX_FWD(CC, GG)                                                                                      \
    raster_fwd_kernel<CC, GG><<<fgrid, kThreads, 0, st>>>(                                                    \
        dc, tiles_x, settings, background, channels, (const float4*)records, hp_records,                      \
        (const int2*)tile_ranges, tile_order, sorted_ids, texture, (int)n_texels, tex_scale, tex_bias, out_img, out_depth, out_reg,     \
        out_alpha, out_tex, out_normal, (float4*)state, ap, nblk, zbuf)
    if (channels == 3 && geo) GSTEX_FWD(3, true);
    else if (channels == 3) GSTEX_FWD(3, false);
    else if (channels == 6 && geo) GSTEX_FWD(6, true);
    else if (channels == 6) GSTEX_FWD(6, false);
    else if (geo) GSTEX_FWD(0, true);
    else GSTEX_FWD(0, false);
#undef GSTEX_FWD
    return launch_status("gstex_raster_fwd");
}

namespace {
int raster_bwd_impl(const gstex_camera* cam, int32_t channels, int32_t settings, const float* background,
                    const float* records, const double* hp_records, const int32_t* tile_ranges, const int32_t* sorted_ids,
                    const int32_t* sorted_slots, const float* texture, int64_t n_texels, float tex_scale,
                    float tex_bias, const float* state, const float* v_img, const float* v_depth, const float* v_reg,
                    const float* v_alpha, const float* v_tex, const float* v_normal, int64_t n_isect, float* partials,
                    uint32_t* row_flags, float* v_texture, void* aux, ZeroBufs zbuf, void* stream) {
    GSTEX_REQUIRE(cam && cam->H > 0 && cam->W > 0, "gstex_raster_bwd: invalid camera");
    GSTEX_REQUIRE(cam->block == kTile, "gstex_raster_bwd: block_width must be %d", kTile);
    GSTEX_REQUIRE(channels >= 1 && channels <= 8, "gstex_raster_bwd: channels must be in [1, 8]");
    int rc = check_settings(settings);
    if (rc) return rc;
    GSTEX_REQUIRE(tile_ranges && state && aux, "gstex_raster_bwd: null pointer (tile_ranges, state and the forward's aux)");
    GSTEX_REQUIRE(n_isect >= 0 && n_isect < (int64_t)INT32_MAX, "gstex_raster_bwd: n_isect out of range");
    GSTEX_REQUIRE(n_isect == 0 || (partials && sorted_ids && sorted_slots), "gstex_raster_bwd: null pair buffer");
    GSTEX_REQUIRE(n_texels >= 0 && n_texels * channels < (int64_t)INT32_MAX, "gstex_raster_bwd: n_texels out of range");
    GSTEX_REQUIRE(n_texels == 0 || (texture && v_texture), "gstex_raster_bwd: null texture");
    GSTEX_REQUIRE(!(settings & GSTEX_SETTING_EVAL_NORMAL) || !v_normal,
                  "gstex_raster_bwd: settings bit 15 (unit-normal eval render) has no normal gradient; pass v_normal = NULL");
    const int tiles_x = (cam->W + kTile - 1) / kTile, tiles_y = (cam->H + kTile - 1) / kTile;
    CamArgs dc = to_device_camera(*cam);
    hipStream_t st = as_stream(stream);
    const AuxLayout al = aux_layout(n_isect, tiles_x * tiles_y, channels);
    const AuxPtrs ap = aux_ptrs(aux, al);
    if (n_isect > 0 && row_flags && hipMemsetAsync(row_flags, 0, (size_t)n_isect * 4, st) != hipSuccess)
        return launch_status("gstex_raster_bwd (row_flags)");
    // costliest units first, from the histogram the forward built (order entries are unit + 1)
    rc = unit_order_from_hist((int32_t)al.n_units, ap.cost, ap.order, ap.order_ws, st);
    if (rc) return rc;
    // depth / distortion / normal gradients present?  (the distortion one only counts when enabled)
    const bool geo = v_depth || v_normal || (v_reg && (settings & GSTEX_SETTING_DIST_REG));
#define GSTEX_BWD(CC, GG)                                                                                      \
    raster_bwd_kernel<CC, GG><<<(unsigned)al.n_units, 64, 0, st>>>(                                            \
        dc, tiles_x, settings, background, channels, (const float4*)records, hp_records,                      \
        (const int2*)tile_ranges, sorted_ids, sorted_slots, texture, (int)n_texels, tex_scale, tex_bias, (const float4*)state,           \
        v_img, v_depth, v_reg, v_alpha, v_tex, v_normal, partials, (unsigned char*)row_flags, v_texture, ap,   \
        zbuf)
    if (channels == 3 && !geo) GSTEX_BWD(3, false);
    else if (channels == 3) GSTEX_BWD(3, true);
    else if (channels == 6 && !geo) GSTEX_BWD(6, false);
    else if (channels == 6) GSTEX_BWD(6, true);
    else if (!geo) GSTEX_BWD(0, false);
    else GSTEX_BWD(0, true);
#undef GSTEX_BWD
    return launch_status("gstex_raster_bwd");
}
}  // namespace

extern "C" int gstex_raster_bwd(const gstex_camera* cam, int32_t channels, int32_t settings,
                                const float* background, const float* records, const double* hp_records,
                                const int32_t* tile_ranges,
                                const int32_t* sorted_ids, const int32_t* sorted_slots,
                                const float* texture, int64_t n_texels, float tex_scale, float tex_bias,
                                const float* state, const float* v_img,
                                const float* v_depth, const float* v_reg, const float* v_alpha, const float* v_tex,
                                const float* v_normal, int64_t n_isect, float* partials, uint32_t* row_flags,
                                float* v_texture, void* aux, void* stream) {
    return raster_bwd_impl(cam, channels, settings, background, records, hp_records, tile_ranges, sorted_ids, sorted_slots,
                           texture, n_texels, tex_scale, tex_bias, state, v_img, v_depth, v_reg, v_alpha, v_tex,
                           v_normal, n_isect, partials, row_flags, v_texture, aux, ZeroBufs{{nullptr, nullptr}, {0, 0}},
                           stream);
}

extern "C" int gstex_raster_bwd_zero(const gstex_camera* cam, int32_t channels, int32_t settings,
                                     const float* background, const float* records, const double* hp_records,
                                     const int32_t* tile_ranges,
                                     const int32_t* sorted_ids, const int32_t* sorted_slots,
                                     const float* texture, int64_t n_texels, float tex_scale, float tex_bias,
                                     const float* state, const float* v_img,
                                     const float* v_depth, const float* v_reg, const float* v_alpha,
                                     const float* v_tex, const float* v_normal, int64_t n_isect, float* partials,
                                     uint32_t* row_flags, float* v_texture, void* aux, float* zero_buf,
                                     int64_t zero_floats, void* stream) {
    GSTEX_REQUIRE(zero_floats >= 0 && (zero_floats == 0 || zero_buf) && zero_buf != v_texture,
                  "gstex_raster_bwd_zero: invalid zero_buf / zero_floats (it must not be the gradient accumulated)");
    return raster_bwd_impl(cam, channels, settings, background, records, hp_records, tile_ranges, sorted_ids, sorted_slots,
                           texture, n_texels, tex_scale, tex_bias, state, v_img, v_depth, v_reg, v_alpha, v_tex,
                           v_normal, n_isect, partials, row_flags, v_texture, aux,
                           ZeroBufs{{zero_floats > 0 ? zero_buf : nullptr, nullptr}, {zero_floats, 0}}, stream);
}

extern "C" size_t gstex_raster_aux_bytes(int64_t n_isect, int32_t n_tiles, int32_t channels) {
    if (n_isect < 0 || n_tiles < 0 || channels < 1 || channels > 8) return 0;
    return aux_layout(n_isect, n_tiles, channels).bytes;
}

template <bool FOLD_AABB>
int setup_bwd_launch(int32_t n, const float* means, const float* scales, float glob_scale, const float* quats,
                     const float* umap, const float* vmap, const int32_t* nth, const int32_t* offsets,
                     float* partials, const uint32_t* row_flags, int32_t rs, int64_t n_rows, const gstex_camera* cam,
                     float* v_means, float* v_scales, float* v_quats, float* v_rgbs, float* v_opacities,
                     float* v_centers, float* v_uv0, hipStream_t st) {
    // no row_flags: the backward accumulated per splat (atomic mode), nothing to sum
    if (row_flags)
        setup_bwd_sum_kernel<<<div_up(n, kSetupBwdRows), 256, 0, st>>>(n, nth, offsets, partials, row_flags, rs, n_rows);
    setup_bwd_chain_kernel<FOLD_AABB><<<div_up(n, 256), 256, 0, st>>>(
        n, means, scales, glob_scale, quats, umap, vmap, nth, offsets, partials, rs, row_flags == nullptr, n_rows,
        to_device_camera(*cam), v_means, v_scales, v_quats, v_rgbs, v_opacities, v_centers, v_uv0);
    return GSTEX_OK;
}

template <bool FOLD_AABB>
int setup_bwd_entry(const char* name, int32_t n, const float* means, const float* scales, float glob_scale,
                    const float* quats, const float* umap, const float* vmap, const int32_t* num_tiles_hit,
                    const int32_t* offsets, float* partials, const uint32_t* row_flags, int32_t row_floats,
                    int64_t n_rows, const gstex_camera* cam, float* v_means, float* v_scales, float* v_quats,
                    float* v_rgbs, float* v_opacities, float* v_centers, float* v_uv0, void* stream) {
    GSTEX_REQUIRE(n >= 0 && cam, "%s: invalid arguments", name);
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(means && scales && quats && umap && vmap && num_tiles_hit && offsets && partials && v_means &&
                      v_scales && v_quats && v_rgbs && v_opacities && v_centers && v_uv0,
                  "%s: null pointer", name);
    GSTEX_REQUIRE(row_floats == kPartRow || row_floats == kPartRowGeo, "%s: row_floats must be %d or %d (got %d)",
                  name, kPartRow, kPartRowGeo, row_floats);
    setup_bwd_launch<FOLD_AABB>(n, means, scales, glob_scale, quats, umap, vmap, num_tiles_hit, offsets, partials,
                                row_flags, row_floats, n_rows, cam, v_means, v_scales, v_quats, v_rgbs, v_opacities,
                                v_centers, v_uv0, as_stream(stream));
    return launch_status(name);
}

extern "C" int gstex_train_epilogue(const gstex_train_epilogue_args* a, void* stream) {
    GSTEX_REQUIRE(a && a->n >= 0, "gstex_train_epilogue: invalid arguments");
    if (a->n == 0) return GSTEX_OK;
    const bool fused = a->sh_degree >= 0 && a->sh_degree <= 4 && a->n_rest >= 0 &&
                       (size_t)kEpiBlock * a->n_rest * 3 * sizeof(float) <= 65536 &&
                       a->n_rest >= (a->sh_degree + 1) * (a->sh_degree + 1) - 1;
    if (!fused) {  // the per-op entry points (an SH layout whose rows do not fit the staging)
        int rc = gstex_raster_setup_bwd_aabb(a->n, a->means, a->scales, 1.0f, a->quats_n, a->opacities, a->umap,
                                             a->vmap, a->num_tiles_hit, a->offsets, a->partials, nullptr, kPartRow,
                                             -1, &a->cam, a->v_means, a->v_scales_act, a->v_quats_n, a->v_rgbs,
                                             a->v_opacities_act, a->v_centers, a->v_uv0, stream);
        if (rc) return rc;
        rc = gstex_sh_rest_bwd(a->n, a->sh_degree, a->n_rest, a->viewdirs, a->v_rgbs, a->v_features_rest, stream);
        if (rc) return rc;
        return gstex_activate_bwd(a->n, a->quats, a->log_scales, a->opacities, a->v_quats_n, a->v_scales_act,
                                  a->v_opacities_act, a->v_quats, a->v_log_scales, a->v_opac_logits, stream);
    }
    GSTEX_REQUIRE(a->means && a->scales && a->quats_n && a->quats && a->log_scales && a->opacities && a->umap &&
                      a->vmap && a->viewdirs && a->num_tiles_hit && a->partials && a->v_means && a->v_quats &&
                      a->v_log_scales && a->v_opac_logits && (a->v_features_rest || a->n_rest == 0) &&
                      a->v_scales_act && a->v_quats_n && a->v_rgbs && a->v_opacities_act && a->v_centers && a->v_uv0,
                  "gstex_train_epilogue: null pointer");
    GSTEX_REQUIRE(((reinterpret_cast<uintptr_t>(a->quats) | reinterpret_cast<uintptr_t>(a->quats_n) |
                    reinterpret_cast<uintptr_t>(a->v_quats) | reinterpret_cast<uintptr_t>(a->v_quats_n) |
                    reinterpret_cast<uintptr_t>(a->partials)) & 15) == 0,
                  "gstex_train_epilogue: quaternion and partial-row buffers must be 16-byte aligned");
    train_epilogue_kernel<<<div_up(a->n, kEpiBlock), kEpiBlock, (size_t)kEpiBlock * a->n_rest * 3 * sizeof(float),
                            as_stream(stream)>>>(
        a->n, a->sh_degree, a->n_rest, to_device_camera(a->cam), a->means, a->scales, a->quats_n, a->quats,
        a->log_scales, a->opacities, a->umap, a->vmap, a->viewdirs, a->num_tiles_hit, a->partials, a->v_means,
        a->v_quats, a->v_log_scales, a->v_opac_logits, a->v_features_rest, a->v_scales_act, a->v_quats_n, a->v_rgbs,
        a->v_opacities_act, a->v_centers, a->v_uv0);
    return launch_status("gstex_train_epilogue");
}

extern "C" int gstex_raster_setup_bwd(int32_t n, const float* means, const float* scales, float glob_scale,
                                      const float* quats, const float* opacities, const float* umap,
                                      const float* vmap, const int32_t* num_tiles_hit, const int32_t* offsets,
                                      float* partials, const uint32_t* row_flags, int32_t row_floats, int64_t n_rows,
                                      const gstex_camera* cam, float* v_means, float* v_scales, float* v_quats,
                                      float* v_rgbs, float* v_opacities, float* v_centers, float* v_uv0, void* stream) {
    (void)opacities;
    return setup_bwd_entry<false>("gstex_raster_setup_bwd", n, means, scales, glob_scale, quats, umap, vmap,
                                  num_tiles_hit, offsets, partials, row_flags, row_floats, n_rows, cam, v_means,
                                  v_scales, v_quats, v_rgbs, v_opacities, v_centers, v_uv0, stream);
}

extern "C" int gstex_raster_setup_bwd_aabb(int32_t n, const float* means, const float* scales, float glob_scale,
                                           const float* quats, const float* opacities, const float* umap,
                                           const float* vmap, const int32_t* num_tiles_hit, const int32_t* offsets,
                                           float* partials, const uint32_t* row_flags, int32_t row_floats,
                                           int64_t n_rows, const gstex_camera* cam, float* v_means, float* v_scales,
                                           float* v_quats, float* v_rgbs, float* v_opacities, float* v_centers,
                                           float* v_uv0, void* stream) {
    (void)opacities;
    return setup_bwd_entry<true>("gstex_raster_setup_bwd_aabb", n, means, scales, glob_scale, quats, umap, vmap,
                                 num_tiles_hit, offsets, partials, row_flags, row_floats, n_rows, cam, v_means,
                                 v_scales, v_quats, v_rgbs, v_opacities, v_centers, v_uv0, stream);
}

extern "C" int gstex_texture_edit(const gstex_camera* cam, int32_t settings, const float* records,
                                  const int32_t* tile_ranges, const int32_t* tile_order, const int32_t* sorted_ids,
                                  const float* edit_rgb, const float* edit_alpha, const float* depth_lo,
                                  const float* depth_hi, int64_t n_texels, float* out, void* stream) {
    GSTEX_REQUIRE(cam && cam->H > 0 && cam->W > 0, "gstex_texture_edit: invalid camera");
    GSTEX_REQUIRE(cam->block == kTile, "gstex_texture_edit: block_width must be %d (got %d)", kTile, cam->block);
    const int known = GSTEX_SETTING_AA_BLUR | GSTEX_SETTING_DIST_REG | GSTEX_SETTING_EDIT | GSTEX_SETTING_EVAL_NORMAL;
    if (settings & ~known) {
        set_error("texture_edit: unsupported settings bits 0x%x", settings & ~known);
        return GSTEX_ERR_UNSUPPORTED;
    }
    GSTEX_REQUIRE(n_texels >= 0, "gstex_texture_edit: n_texels < 0");
    GSTEX_REQUIRE(tile_ranges && edit_rgb && edit_alpha && depth_lo && depth_hi && (out || n_texels == 0),
                  "gstex_texture_edit: null pointer");
    const int tiles_x = (cam->W + kTile - 1) / kTile, tiles_y = (cam->H + kTile - 1) / kTile;
    CamArgs dc = to_device_camera(*cam);
    texture_edit_kernel<<<tiles_x * tiles_y, kThreads, 0, as_stream(stream)>>>(
        dc, tiles_x, settings, (const float4*)records, (const int2*)tile_ranges, tile_order, sorted_ids, edit_rgb,
        edit_alpha, depth_lo, depth_hi, (int)n_texels, out);
    return launch_status("gstex_texture_edit");
}
