// splat_math.h — per-splat device functions shared by the per-op kernels and the training prologue's fused
// kernels (trainstep.hip): the parameter activations (activations.hip), the preprocessing (preprocess.hip), the SH
// colour (sh_texture.hip) and the block scans (binning.hip).  Each per-op kernel and the fused kernel call the same
// function on the same fp32 values (-ffp-contract=off: every operation individually rounded), so their outputs are
// bit-identical (tests/test_gpu_fused.py).
#pragma once

#include "gstex_common.h"

namespace gstex {

// ---- activations: gstex.py:1059-1066, 975-990, 1101-1104 (see activations.hip) ----------------------------------
__device__ __forceinline__ float act_norm4(float a, float b, float c, float d) {
    return sqrtf(((a * a + b * b) + c * c) + d * d);
}

struct Activated {
    float q[4];          // quats / |quats|
    float s0, s1, s2;    // scales (the third: 1e-5 * mean of the first two, detached)
    float opacity;
    float um[3], vm[3];  // umap, vmap (get_uv_mapping of the re-normalised quaternion)
    float vd[3];         // viewdirs
};

__device__ __forceinline__ Activated activate_splat(float4 q, float ls0, float ls1, float logit, float m0, float m1,
                                                    float mx, float my, float mz, const float* campos) {
    Activated a;
    const float nq = act_norm4(q.x, q.y, q.z, q.w);
    const float w = q.x / nq, x = q.y / nq, y = q.z / nq, z = q.w / nq;
    a.q[0] = w; a.q[1] = x; a.q[2] = y; a.q[3] = z;
    a.s0 = fmaxf(expf(ls0), 1e-9f);
    a.s1 = fmaxf(expf(ls1), 1e-9f);
    a.s2 = 1e-5f * ((a.s0 + a.s1) / 2.0f);
    a.opacity = 1.0f / (1.0f + expf(-logit));
    // get_uv_mapping: rotation of the re-normalised quaternion (F.normalize, eps 1e-12)
    const float n2 = fmaxf(act_norm4(w, x, y, z), 1e-12f);
    const float rw = w / n2, rx = x / n2, ry = y / n2, rz = z / n2;
    a.um[0] = m0 * (1.0f - 2.0f * (ry * ry + rz * rz));
    a.um[1] = m0 * (2.0f * (rx * ry + rw * rz));
    a.um[2] = m0 * (2.0f * (rx * rz - rw * ry));
    a.vm[0] = m1 * (2.0f * (rx * ry - rw * rz));
    a.vm[1] = m1 * (1.0f - 2.0f * (rx * rx + rz * rz));
    a.vm[2] = m1 * (2.0f * (ry * rz + rw * rx));
    const float dx = mx - campos[0], dy = my - campos[1], dz = mz - campos[2];
    const float nd = sqrtf((dx * dx + dy * dy) + dz * dz);
    a.vd[0] = dx / nd;
    a.vd[1] = dy / nd;
    a.vd[2] = dz / nd;
    return a;
}

__device__ __forceinline__ void store_activated(int i, const Activated& a, float* quats_n, float* scales,
                                                float* opacities, float* uv0, float* umap, float* vmap,
                                                float* viewdirs) {
    reinterpret_cast<float4*>(quats_n)[i] = make_float4(a.q[0], a.q[1], a.q[2], a.q[3]);
    scales[3 * i] = a.s0;
    scales[3 * i + 1] = a.s1;
    scales[3 * i + 2] = a.s2;
    opacities[i] = a.opacity;
    umap[3 * i] = a.um[0];
    umap[3 * i + 1] = a.um[1];
    umap[3 * i + 2] = a.um[2];
    vmap[3 * i] = a.vm[0];
    vmap[3 * i + 1] = a.vm[1];
    vmap[3 * i + 2] = a.vm[2];
    uv0[2 * i] = 0.5f;
    uv0[2 * i + 1] = 0.5f;
    viewdirs[3 * i] = a.vd[0];
    viewdirs[3 * i + 1] = a.vd[1];
    viewdirs[3 * i + 2] = a.vd[2];
}

// the activations' backward (activations.hip): the quaternion normalisation, exp with the clamp mask for the first two
// scale axes (the third is detached) and the sigmoid
__device__ __forceinline__ void activate_bwd_splat(float4 q, float ls0, float ls1, float o, float4 g, float gs0,
                                                   float gs1, float go, float4& vq, float& vls0, float& vls1,
                                                   float& vo) {
    const float nq = act_norm4(q.x, q.y, q.z, q.w);
    const float w = q.x / nq, x = q.y / nq, y = q.z / nq, z = q.w / nq;
    const float d = ((w * g.x + x * g.y) + y * g.z) + z * g.w;
    vq = make_float4((g.x - w * d) / nq, (g.y - x * d) / nq, (g.z - y * d) / nq, (g.w - z * d) / nq);
    const float e0 = expf(ls0), e1 = expf(ls1);
    vls0 = (e0 >= 1e-9f) ? gs0 * e0 : 0.0f;
    vls1 = (e1 >= 1e-9f) ? gs1 * e1 : 0.0f;
    vo = go * ((1.0f - o) * o);
}

// ---- preprocessing: project_points' depth, get_aabb_2d, get_num_tiles_hit_2d (gstex.py:1077-1080) ---------------
struct Preprocessed {
    float depth, cx, cy, ex, ey;
    int nth;
};

__device__ __forceinline__ Homog splat_homog(const Camera& cam, f3 mu, float s0, float s1, float glob, const float* q4,
                                             Frame& fr, float& su, float& sv) {
    fr = quat_frame(q4);
    su = s0 * glob;
    sv = s1 * glob;
    return splat_homography(cam, mu, su, sv, fr);
}

__device__ __forceinline__ Preprocessed preprocess_splat(const Camera& cam, f3 mu, float s0, float s1, float glob,
                                                         const float* q4, int tiles_x, int tiles_y, int block) {
    Preprocessed p;
    p.depth = vrow(cam, 2, mu) + cam.V[11];
    Frame fr;
    float su, sv;
    Homog h = splat_homog(cam, mu, s0, s1, glob, q4, fr, su, sv);
    p.cx = 0.0f; p.cy = 0.0f; p.ex = 0.0f; p.ey = 0.0f;
    if (!aabb_from_homog(h, p.cx, p.cy, p.ex, p.ey)) { p.cx = p.cy = p.ex = p.ey = 0.0f; }
    Rect r = tile_rect(p.cx, p.cy, p.ex, p.ey, tiles_x, tiles_y, block);
    p.nth = (r.x1 - r.x0) * (r.y1 - r.y0);
    return p;
}

// ---- the splat's raster record (raster.hip setup_kernel, gstex_raster_setup) ---------------------------------------
// Evaluated in fp64 and rounded once per value (one thread per splat, ~100 fp64 operations): its fp32 evaluation was
// the dominant error of the means / quats gradients (tools/grad_precision.py).  Inputs are the splat's
// fp32 values (the activated scales / quaternion, its colour, opacity, AABB centre, UV frame and texel block dims).
__device__ __forceinline__ void splat_record(const Camera& cam, float mx, float my, float mz, float s0, float s1,
                                             float glob, const float* q4, const float* rgb, float opac, float cx,
                                             float cy, const float* uv0, const float* um3, const float* vm3,
                                             const int32_t* td, float* __restrict__ rec_out,
                                             double* __restrict__ hp_out = nullptr) {
    const FrameT<double> fr = quat_frame_t<double>(q4);
    const double su = (double)s0 * (double)glob, sv = (double)s1 * (double)glob;
    const d3 mu = d3{(double)mx, (double)my, (double)mz};
    const AnchoredT<double> h = splat_anchored(cam, mu, su, sv, fr);
    const d3 dir = d3{(double)cam.campos[0] - mu.x, (double)cam.campos[1] - mu.y, (double)cam.campos[2] - mu.z};
    const double sgn = dot3(fr.tw, dir) < 0.0 ? -1.0 : 1.0;
    const d3 um = d3{(double)um3[0], (double)um3[1], (double)um3[2]};
    const d3 vm = d3{(double)vm3[0], (double)vm3[1], (double)vm3[2]};
    float r[GSTEX_REC_FLOATS];
    const AffineHomogT<double> ah = affine_homog(h.Tu, h.Tv, h.Tw);
    r[R_A + 0] = (float)ah.A.x; r[R_A + 1] = (float)ah.A.y; r[R_A + 2] = (float)ah.A.z;
    r[R_B + 0] = (float)ah.B.x; r[R_B + 1] = (float)ah.B.y; r[R_B + 2] = (float)ah.B.z;
    r[R_PZ] = (float)ah.Pz;
    r[R_TW + 0] = (float)h.Tw.x; r[R_TW + 1] = (float)h.Tw.y; r[R_TW + 2] = (float)h.Tw.z;
    r[R_XY + 0] = cx; r[R_XY + 1] = cy;
    r[R_OPAC] = opac;
    if (hp_out) {
        // near edge-on (gstex_common.h kHpCos): the fp64 row for the backward, flagged by the opacity's sign bit
        const double dn = sqrt(dot3(dir, dir));
        if (fabs(dot3(fr.tw, dir)) < kHpCos * dn) {
            r[R_OPAC] = -opac;
            const double v[H_FIELDS] = {ah.A.x, ah.A.y, ah.A.z, ah.B.x, ah.B.y, ah.B.z, ah.Pz, h.xa, h.ya,
                                        h.Tw.x, h.Tw.y, h.Tw.z};
#pragma unroll
            for (int k = 0; k < H_FIELDS; ++k) hp_out[k] = v[k];
        }
    }
    r[R_RGB + 0] = rgb[0]; r[R_RGB + 1] = rgb[1]; r[R_RGB + 2] = rgb[2];
    r[R_NRM + 0] = (float)(sgn * fr.tw.x); r[R_NRM + 1] = (float)(sgn * fr.tw.y); r[R_NRM + 2] = (float)(sgn * fr.tw.z);
    // the texture affine in texel units: the sample point (tu h, tv w) = (tu0 + auu u + auv v) h, ... is read as
    // fma(u, auu h, fma(v, auv h, tu0 h)) -- two fused multiply-adds per coordinate instead of three operations
    const double hd = (double)td[0], wd = (double)td[1];
    r[R_TU0] = (float)((double)uv0[0] * hd);
    r[R_AUU] = (float)(su * dot3(fr.tu, um) * hd);
    r[R_AUV] = (float)(sv * dot3(fr.tv, um) * hd);
    r[R_TV0] = (float)((double)uv0[1] * wd);
    r[R_AVU] = (float)(su * dot3(fr.tu, vm) * wd);
    r[R_AVV] = (float)(sv * dot3(fr.tv, vm) * wd);
    r[R_H] = __int_as_float(td[0]);
    r[R_W] = __int_as_float(td[1]);
    r[R_OFF] = __int_as_float(td[2]);
    r[R_XA] = (float)h.xa;
    r[R_YA] = (float)h.ya;
    r[R_HM1] = (float)(td[0] - 1);
    r[R_WM1] = (float)(td[1] - 1);
    float4* dst = reinterpret_cast<float4*>(rec_out);
#pragma unroll
    for (int k = 0; k < GSTEX_REC_FLOATS / 4; ++k) dst[k] = make_float4(r[4 * k], r[4 * k + 1], r[4 * k + 2], r[4 * k + 3]);
}

// ---- SH colour of the gsplat-0.1 lineage, degree <= 4 (see sh_texture.hip) -----------------------------------------
namespace {
constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
__constant__ float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
__constant__ float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f,  -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};
__constant__ float SH_C4[9] = {2.5033429417967046f,  -1.7701307697799304f, 0.9461746957575601f,
                               -0.6690465435572892f, 0.10578554691520431f, -0.6690465435572892f,
                               0.47308734787878004f, -1.7701307697799304f, 0.6258357354491761f};
}  // namespace

// basis[k] for k < (degree+1)^2
__device__ __forceinline__ void sh_basis(int degree, float x, float y, float z, float* b) {
    b[0] = SH_C0;
    if (degree < 1) return;
    float nrm = sqrtf((x * x + y * y) + z * z);
    x = x / nrm; y = y / nrm; z = z / nrm;
    b[1] = -SH_C1 * y;
    b[2] = SH_C1 * z;
    b[3] = -SH_C1 * x;
    if (degree < 2) return;
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    b[4] = SH_C2[0] * xy;
    b[5] = SH_C2[1] * yz;
    b[6] = SH_C2[2] * ((2.0f * zz - xx) - yy);
    b[7] = SH_C2[3] * xz;
    b[8] = SH_C2[4] * (xx - yy);
    if (degree < 3) return;
    b[9] = SH_C3[0] * y * (3.0f * xx - yy);
    b[10] = SH_C3[1] * xy * z;
    b[11] = SH_C3[2] * y * ((4.0f * zz - xx) - yy);
    b[12] = SH_C3[3] * z * ((2.0f * zz - 3.0f * xx) - 3.0f * yy);
    b[13] = SH_C3[4] * x * ((4.0f * zz - xx) - yy);
    b[14] = SH_C3[5] * z * (xx - yy);
    b[15] = SH_C3[6] * x * (xx - 3.0f * yy);
    if (degree < 4) return;
    b[16] = SH_C4[0] * xy * (xx - yy);
    b[17] = SH_C4[1] * yz * (3.0f * xx - yy);
    b[18] = SH_C4[2] * xy * (7.0f * zz - 1.0f);
    b[19] = SH_C4[3] * yz * (7.0f * zz - 3.0f);
    b[20] = SH_C4[4] * (zz * (35.0f * zz - 30.0f) + 3.0f);
    b[21] = SH_C4[5] * xz * (7.0f * zz - 3.0f);
    b[22] = SH_C4[6] * (xx - yy) * (7.0f * zz - 1.0f);
    b[23] = SH_C4[7] * xz * (xx - 3.0f * yy);
    b[24] = SH_C4[8] * (xx * (xx - 3.0f * yy) - yy * (3.0f * xx - yy));
}

// colour = sum_{k0 <= k < (degree+1)^2} basis[k] * c[k] (c: the splat's coefficient row, indexed from basis 0;
// k0 = 1 for the rest coefficients, the DC term zeroed by the caller, gstex.py:1100)
__device__ __forceinline__ void sh_colour(int degree, int k0, float dx, float dy, float dz, const float* c, float& r0,
                                          float& r1, float& r2) {
    float b[25];
    sh_basis(degree, dx, dy, dz, b);
    const int nb = (degree + 1) * (degree + 1);
    r0 = 0.f; r1 = 0.f; r2 = 0.f;
    for (int k = k0; k < nb; ++k) {
        r0 = r0 + b[k] * c[3 * k];
        r1 = r1 + b[k] * c[3 * k + 1];
        r2 = r2 + b[k] * c[3 * k + 2];
    }
}

// the coefficient gradient row of one splat: row[3 k + c] = basis[k + k0] * g_c for k < K (0 past the degree)
__device__ __forceinline__ void sh_grad_row(int degree, int k0, int K, float dx, float dy, float dz, float g0,
                                            float g1, float g2, float* row) {
    float b[25];
    sh_basis(degree, dx, dy, dz, b);
    const int nb = (degree + 1) * (degree + 1);
    for (int k = 0; k < K; ++k) {
        const float bk = (k + k0 < nb) ? b[k + k0] : 0.0f;
        row[3 * k] = bk * g0;
        row[3 * k + 1] = bk * g1;
        row[3 * k + 2] = bk * g2;
    }
}

// A workgroup's contiguous span of coefficient rows copied between global memory and LDS with consecutive lanes on
// consecutive words (16-B vectors, several in flight per thread, when both sides are 16-B aligned).
template <int kThreads>
__device__ __forceinline__ void sh_copy_span(float* __restrict__ dst, const float* __restrict__ src, int total) {
    const int t = threadIdx.x;
    int done = 0;
    if ((((uintptr_t)src | (uintptr_t)dst) & 15u) == 0) {
        const int n4 = total >> 2;
        const float4* s4 = reinterpret_cast<const float4*>(src);
        float4* d4 = reinterpret_cast<float4*>(dst);
#pragma unroll 4
        for (int q = t; q < n4; q += kThreads) d4[q] = s4[q];
        done = n4 << 2;
    }
    for (int q = done + t; q < total; q += kThreads) dst[q] = src[q];
}

// ---- block scans (binning.hip) --------------------------------------------------------------------------------------
// Inclusive wave64 scan.
__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// Exclusive scan of one kThreads-thread block's per-thread values; returns the block total in *total.
template <int kThreads>
__device__ __forceinline__ int block_excl_scan(int v, int* s_wave, int* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = wave_incl_scan(v);
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    int wave_off = 0, sum = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) {
        int s = s_wave[w];
        if (w < wave) wave_off += s;
        sum += s;
    }
    __syncthreads();
    *total = sum;
    return wave_off + incl - v;
}

// Pair-capacity guard (gstex_scan_offsets_guarded, ABI 13), applied by the thread that writes the total out[n]: the
// step's overflow flag (1.0f when the total exceeds the pair buffers' capacity; the first render of a step writes it,
// later ones OR into it) and, when given, the total in device-writable host memory (no copy, no synchronisation:
// the host polls the word, which it set to a sentinel before the launch).  Plain vector stores.
struct ScanGuard {
    long long capacity;
    float* flag;
    int32_t* host_count;
    int first;
};
__device__ __forceinline__ void apply_guard(const ScanGuard& g, int total) {
    if (g.flag) {
        const float over = (long long)total > g.capacity ? 1.0f : 0.0f;
        *g.flag = g.first ? over : fmaxf(*g.flag, over);
    }
    if (g.host_count) {
        *g.host_count = total;
        __threadfence_system();  // the host polls this word (ops.PairCapacity): no event marks the scan's end
    }
}

}  // namespace gstex
