// gstex_common.h — device math shared by every gfx950 kernel of libgstex_hip.so.
//
// The fp32 operation ORDER in this file is part of the numerical contract: oracle/raster.py
// restates each function below op-for-op (the library is compiled with -ffp-contract=off, so no
// fused multiply-adds are formed), which is what makes the threshold decisions of the composite
// (alpha >= 1/255, T < 1e-4, z >= near) agree between the GPU and the CPU oracle, except within a few ulps of a
// threshold: the rasterizer's pair evaluation uses the hardware v_exp_f32 / v_rcp_f32 (raster.hip eval_hit,
// GSTEX_FAST_EVAL), and the tests tell such flips apart by the oracle's decision margins.
//
// Semantics follow the call-site contracts of the reference (nerfstudio/models/gstex.py) and the
// 2DGS formulation its argument list implies.  Pixel (x, y) is evaluated at its
// centre (x + 0.5, y + 0.5): the reference's own depths_to_points (gstex.py:138-139) maps rendered pixel
// (i, j) to the ray through ((j + 0.5 - cx) / fx, (i + 0.5 - cy) / fy), which its normal loss compares
// with the rendered normal (gstex.py:1219, 1313); 2DGS, whose depths_to_points has no +0.5, evaluates at
// the integer point instead (lineage table).

#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gstex_hip.h"

namespace gstex {

constexpr int kTile = 16;               // BLOCK_WIDTH, gstex.py:1075
constexpr int kTilePixels = kTile * kTile;
constexpr float kCutoff2 = 9.0f;        // 3-sigma AABB cutoff (2DGS compute_aabb)
constexpr float kMinExtent = 2.1213180f;// cutoff * FilterSize (3 * 0.707106)
constexpr float kNear = 0.2f;           // 2DGS near_n
constexpr float kFarRatio = 100.0f / 99.8f;  // far_n / (far_n - near_n), rounded to fp32 once
constexpr float kAlphaMax = 0.99f;
constexpr float kAlphaMin = 1.0f / 255.0f;
constexpr float kTMin = 1e-4f;
constexpr float kFilterInvSq = 2.0f;    // 2DGS FilterInvSquare
constexpr float kProjClip = 0.01f;      // project_points near clip (gsplat-0.1 clip_thresh)

// Kernel argument form of gstex_camera (device pointers + scalars).
struct CamArgs {
    const float* viewmat;
    const float* c2w;
    float fx, fy, cx, cy;
    int H, W, block;
};

__host__ inline CamArgs to_device_camera(const gstex_camera& c) {
    CamArgs d;
    d.viewmat = c.viewmat; d.c2w = c.c2w;
    d.fx = c.fx; d.fy = c.fy; d.cx = c.cx; d.cy = c.cy;
    d.H = c.H; d.W = c.W; d.block = c.block;
    return d;
}

// In-kernel camera: the 12 view-matrix words are wave-uniform loads (scalar cache).
struct Camera {
    float V[12];
    float campos[3];
    float fx, fy, cx, cy;
    int H, W, block;
};

__device__ __forceinline__ Camera load_camera(const CamArgs& a) {
    Camera c;
#pragma unroll
    for (int i = 0; i < 12; ++i) c.V[i] = a.viewmat[i];
    if (a.c2w) {
        c.campos[0] = a.c2w[3]; c.campos[1] = a.c2w[7]; c.campos[2] = a.c2w[11];
    } else {  // -R^T t
        c.campos[0] = -((c.V[0] * c.V[3] + c.V[4] * c.V[7]) + c.V[8] * c.V[11]);
        c.campos[1] = -((c.V[1] * c.V[3] + c.V[5] * c.V[7]) + c.V[9] * c.V[11]);
        c.campos[2] = -((c.V[2] * c.V[3] + c.V[6] * c.V[7]) + c.V[10] * c.V[11]);
    }
    c.fx = a.fx; c.fy = a.fy; c.cx = a.cx; c.cy = a.cy;
    c.H = a.H; c.W = a.W; c.block = a.block;
    return c;
}

// 3-vectors and the per-splat geometry, templated on the arithmetic type: float for the per-pixel work and the
// preprocessing kernels, double for the raster's per-splat record (setup) and its backward chain (setup_bwd), whose
// fp32 rounding was measured to dominate the means / quats gradient error (tools/grad_precision.py).
template <typename T> struct V3 { T x, y, z; };
using f3 = V3<float>;
using d3 = V3<double>;

__device__ __forceinline__ f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
template <typename T> __device__ __forceinline__ T dot3(V3<T> a, V3<T> b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
template <typename T> __device__ __forceinline__ V3<T> cross3(V3<T> a, V3<T> b) {
    return V3<T>{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
template <typename T> __device__ __forceinline__ V3<T> scale3(V3<T> a, T s) { return V3<T>{a.x * s, a.y * s, a.z * s}; }
template <typename T> __device__ __forceinline__ V3<T> add3(V3<T> a, V3<T> b) { return V3<T>{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ d3 to_d3(f3 a) { return d3{(double)a.x, (double)a.y, (double)a.z}; }
__device__ __forceinline__ f3 to_f3(d3 a) { return f3{(float)a.x, (float)a.y, (float)a.z}; }

// Normalised wxyz quaternion -> rotation columns (t_u, t_v, t_w).  Matches
// nerfstudio/utils/rotations.py:43-72 on unit quaternions (wxyz, real part first).
template <typename T> struct FrameT { V3<T> tu, tv, tw; T qw, qx, qy, qz, qnorm; };
using Frame = FrameT<float>;

template <typename T>
__device__ __forceinline__ FrameT<T> quat_frame_t(const float* q4) {
    FrameT<T> f;
    T w = q4[0], x = q4[1], y = q4[2], z = q4[3];
    T nrm = sqrt(((w * w + x * x) + y * y) + z * z);
    w = w / nrm; x = x / nrm; y = y / nrm; z = z / nrm;
    f.qw = w; f.qx = x; f.qy = y; f.qz = z; f.qnorm = nrm;
    const T one = 1, two = 2;
    T r00 = one - two * (y * y + z * z);
    T r01 = two * (x * y - w * z);
    T r02 = two * (x * z + w * y);
    T r10 = two * (x * y + w * z);
    T r11 = one - two * (x * x + z * z);
    T r12 = two * (y * z - w * x);
    T r20 = two * (x * z - w * y);
    T r21 = two * (y * z + w * x);
    T r22 = one - two * (x * x + y * y);
    f.tu = V3<T>{r00, r10, r20};
    f.tv = V3<T>{r01, r11, r21};
    f.tw = V3<T>{r02, r12, r22};
    return f;
}
__device__ __forceinline__ Frame quat_frame(const float* q4) { return quat_frame_t<float>(q4); }

// Row r of the 3x3 rotation part of the view matrix applied to a vector.
template <typename T>
__device__ __forceinline__ T vrow(const Camera& c, int r, V3<T> a) {
    return ((T)c.V[4 * r + 0] * a.x + (T)c.V[4 * r + 1] * a.y) + (T)c.V[4 * r + 2] * a.z;
}

// Splat -> pixel homogeneous matrix M = K [R|t] [[su t_u, sv t_v, mu],[0,0,1]] (rows Tu,Tv,Tw).
template <typename T> struct HomogT { V3<T> Tu, Tv, Tw; };
using Homog = HomogT<float>;

template <typename T>
__device__ __forceinline__ HomogT<T> splat_homography(const Camera& c, V3<T> mu, T su, T sv, const FrameT<T>& fr) {
    V3<T> a = scale3(fr.tu, su);
    V3<T> b = scale3(fr.tv, sv);
    T W0[3], W1[3], W2[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        W0[r] = vrow(c, r, a);
        W1[r] = vrow(c, r, b);
        W2[r] = vrow(c, r, mu) + (T)c.V[4 * r + 3];
    }
    const T fx = c.fx, fy = c.fy, cx = c.cx, cy = c.cy;
    HomogT<T> h;
    h.Tu = V3<T>{fx * W0[0] + cx * W0[2], fx * W1[0] + cx * W1[2], fx * W2[0] + cx * W2[2]};
    h.Tv = V3<T>{fy * W0[1] + cy * W0[2], fy * W1[1] + cy * W1[2], fy * W2[1] + cy * W2[2]};
    h.Tw = V3<T>{W0[2], W1[2], W2[2]};
    return h;
}

// dL/dM -> dL/d(mu, su, sv, t_u, t_v)
template <typename T> struct HomogGradT { V3<T> dmu; T dsu, dsv; V3<T> dtu, dtv; };
using HomogGrad = HomogGradT<float>;

// R_cw^T e (the view matrix's rotation transposed)
template <typename T>
__device__ __forceinline__ V3<T> view_rt(const Camera& c, T e0, T e1, T e2) {
    return V3<T>{((T)c.V[0] * e0 + (T)c.V[4] * e1) + (T)c.V[8] * e2, ((T)c.V[1] * e0 + (T)c.V[5] * e1) + (T)c.V[9] * e2,
                 ((T)c.V[2] * e0 + (T)c.V[6] * e1) + (T)c.V[10] * e2};
}

template <typename T>
__device__ __forceinline__ HomogGradT<T> splat_homography_vjp(const Camera& c, T su, T sv, const FrameT<T>& fr,
                                                              V3<T> dTu, V3<T> dTv, V3<T> dTw) {
    // W rows: dW[0,:] = fx dTu, dW[1,:] = fy dTv, dW[2,:] = cx dTu + cy dTv + dTw
    V3<T> dW0r = scale3(dTu, (T)c.fx);
    V3<T> dW1r = scale3(dTv, (T)c.fy);
    V3<T> dW2r = add3(add3(scale3(dTu, (T)c.cx), scale3(dTv, (T)c.cy)), dTw);
    // columns of dW: col k = (dW0r[k], dW1r[k], dW2r[k]); d(vec) = R_cw^T col
    V3<T> da = view_rt(c, dW0r.x, dW1r.x, dW2r.x);
    V3<T> db = view_rt(c, dW0r.y, dW1r.y, dW2r.y);
    HomogGradT<T> g;
    g.dmu = view_rt(c, dW0r.z, dW1r.z, dW2r.z);
    g.dsu = dot3(fr.tu, da);
    g.dsv = dot3(fr.tv, db);
    g.dtu = scale3(da, su);
    g.dtv = scale3(db, sv);
    return g;
}

// Anchored form of the same homography, used by the rasterizer.  With the anchor (xa, ya) = the
// projection of the splat centre, k = px*Tw - Tu is evaluated as (px - xa)*Tw - (Tu - xa*Tw): the
// z-component of Tu - xa*Tw is exactly 0 and nothing of size |px*Tw| is ever cancelled, which is
// what keeps the fp32 forward and especially the backward (means / quats gradients) accurate.
//   Tu' = Tu - xa Tw = fx (W0[0] - xn W0[2], W1[0] - xn W1[2], 0),   xn = W2[0] / W2[2]
//   Tv' = Tv - ya Tw = fy (W0[1] - yn W0[2], W1[1] - yn W1[2], 0),   yn = W2[1] / W2[2]
//   xa = fx xn + cx,  ya = fy yn + cy
template <typename T> struct AnchoredT { V3<T> Tu, Tv, Tw; T xn, yn, xa, ya; };

template <typename T>
__device__ __forceinline__ AnchoredT<T> splat_anchored(const Camera& c, V3<T> mu, T su, T sv, const FrameT<T>& fr) {
    V3<T> a = scale3(fr.tu, su);
    V3<T> b = scale3(fr.tv, sv);
    T W0[3], W1[3], W2[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        W0[r] = vrow(c, r, a);
        W1[r] = vrow(c, r, b);
        W2[r] = vrow(c, r, mu) + (T)c.V[4 * r + 3];
    }
    const T fx = c.fx, fy = c.fy, cx = c.cx, cy = c.cy;
    AnchoredT<T> h;
    h.xn = W2[0] / W2[2];
    h.yn = W2[1] / W2[2];
    h.Tu = V3<T>{fx * (W0[0] - h.xn * W0[2]), fx * (W1[0] - h.xn * W1[2]), (T)0};
    h.Tv = V3<T>{fy * (W0[1] - h.yn * W0[2]), fy * (W1[1] - h.yn * W1[2]), (T)0};
    h.Tw = V3<T>{W0[2], W1[2], W2[2]};
    h.xa = fx * h.xn + cx;
    h.ya = fy * h.yn + cy;
    return h;
}

// Gradient of the anchored form w.r.t. (mu, su, sv, t_u, t_v), treating the anchor as a constant
// (k and l do not depend on it).  A = dL/dTu, B = dL/dTv, Pw = dL/dTw accumulated with the
// anchored pixel offsets:  dW[0,:] = fx A,  dW[1,:] = fy B,  dW[2,:] = Pw - xn dW[0,:] - yn dW[1,:].
template <typename T>
__device__ __forceinline__ HomogGradT<T> splat_anchored_vjp(const Camera& c, T su, T sv, const FrameT<T>& fr, T xn,
                                                            T yn, V3<T> A, V3<T> B, V3<T> Pw) {
    V3<T> dW0r = scale3(A, (T)c.fx);
    V3<T> dW1r = scale3(B, (T)c.fy);
    V3<T> dW2r = V3<T>{(Pw.x - xn * dW0r.x) - yn * dW1r.x, (Pw.y - xn * dW0r.y) - yn * dW1r.y,
                       (Pw.z - xn * dW0r.z) - yn * dW1r.z};
    V3<T> da = view_rt(c, dW0r.x, dW1r.x, dW2r.x);
    V3<T> db = view_rt(c, dW0r.y, dW1r.y, dW2r.y);
    HomogGradT<T> g;
    g.dmu = view_rt(c, dW0r.z, dW1r.z, dW2r.z);
    g.dsu = dot3(fr.tu, da);
    g.dsv = dot3(fr.tv, db);
    g.dtu = scale3(da, su);
    g.dtv = scale3(db, sv);
    return g;
}

// dL/d(rotation columns) -> dL/d(raw quaternion), through the normalisation.
template <typename T>
__device__ __forceinline__ void frame_vjp(const FrameT<T>& f, V3<T> dtu, V3<T> dtv, V3<T> dtw, T* dq) {
    const T w = f.qw, x = f.qx, y = f.qy, z = f.qz;
    const T two = 2;
    // R[r][c]: column c = (tu, tv, tw)[c], row r = component
    const T d00 = dtu.x, d10 = dtu.y, d20 = dtu.z;
    const T d01 = dtv.x, d11 = dtv.y, d21 = dtv.z;
    const T d02 = dtw.x, d12 = dtw.y, d22 = dtw.z;
    T gw = two * (-z * d01 + y * d02 + z * d10 - x * d12 - y * d20 + x * d21);
    T gx = two * (y * d01 + z * d02 + y * d10 - two * x * d11 - w * d12 + z * d20 + w * d21 - two * x * d22);
    T gy = two * (-two * y * d00 + x * d01 + w * d02 + x * d10 + z * d12 - w * d20 + z * d21 - two * y * d22);
    T gz = two * (-two * z * d00 - w * d01 + x * d02 + w * d10 - two * z * d11 + y * d12 + x * d20 + y * d21);
    T proj = ((w * gw + x * gx) + y * gy) + z * gz;
    T inv = (T)1 / f.qnorm;
    dq[0] = (gw - w * proj) * inv;
    dq[1] = (gx - x * proj) * inv;
    dq[2] = (gy - y * proj) * inv;
    dq[3] = (gz - z * proj) * inv;
}

// 2DGS compute_aabb (3-sigma disc) -> screen centre + per-axis half extent.  Returns false when
// the splat must be culled (centre at/behind the near plane, or the disc crosses the camera
// plane: d >= 0).
__device__ __forceinline__ bool aabb_from_homog(const Homog& h, float& cxo, float& cyo,
                                                float& exo, float& eyo) {
    const f3 Tu = h.Tu, Tv = h.Tv, Tw = h.Tw;
    if (!(Tw.z > kNear)) return false;
    float d = (kCutoff2 * (Tw.x * Tw.x) + kCutoff2 * (Tw.y * Tw.y)) - Tw.z * Tw.z;
    if (!(d < 0.0f)) return false;
    float fxy = kCutoff2 / d;
    float fz = -1.0f / d;
    float px = (fxy * (Tu.x * Tw.x) + fxy * (Tu.y * Tw.y)) + fz * (Tu.z * Tw.z);
    float py = (fxy * (Tv.x * Tw.x) + fxy * (Tv.y * Tw.y)) + fz * (Tv.z * Tw.z);
    float qx = (fxy * (Tu.x * Tu.x) + fxy * (Tu.y * Tu.y)) + fz * (Tu.z * Tu.z);
    float qy = (fxy * (Tv.x * Tv.x) + fxy * (Tv.y * Tv.y)) + fz * (Tv.z * Tv.z);
    float hx = px * px - qx;
    float hy = py * py - qy;
    float ex = sqrtf(fmaxf(1e-4f, hx));
    float ey = sqrtf(fmaxf(1e-4f, hy));
    cxo = px; cyo = py;
    exo = fmaxf(ex, kMinExtent);
    eyo = fmaxf(ey, kMinExtent);
    return true;
}

// dL/d(AABB centre) -> dL/d(homography rows) through aabb_from_homog's centre (the extents carry no gradient:
// they only bound the tile lists).  c = (9 (T.x Tw.x + T.y Tw.y) - T.z Tw.z) / d for T = Tu (x) and Tv (y).
__device__ __forceinline__ void aabb_centre_vjp(const Homog& h, float cx, float cy, float gcx, float gcy, f3& dTu,
                                                f3& dTv, f3& dTw) {
    const f3 Tu = h.Tu, Tv = h.Tv, Tw = h.Tw;
    float d = (kCutoff2 * (Tw.x * Tw.x) + kCutoff2 * (Tw.y * Tw.y)) - Tw.z * Tw.z;
    float invd = 1.0f / d;
    dTu = scale3(f3{kCutoff2 * Tw.x, kCutoff2 * Tw.y, -Tw.z}, gcx * invd);
    dTv = scale3(f3{kCutoff2 * Tw.x, kCutoff2 * Tw.y, -Tw.z}, gcy * invd);
    f3 dd = f3{2.0f * kCutoff2 * Tw.x, 2.0f * kCutoff2 * Tw.y, -2.0f * Tw.z};
    dTw = add3(scale3(add3(f3{kCutoff2 * Tu.x, kCutoff2 * Tu.y, -Tu.z}, scale3(dd, -cx)), gcx * invd),
               scale3(add3(f3{kCutoff2 * Tv.x, kCutoff2 * Tv.y, -Tv.z}, scale3(dd, -cy)), gcy * invd));
}

// Tile rectangle [x0,x1) x [y0,y1) in tile units (gsplat-0.1 get_tile_bbox convention).
struct Rect { int x0, x1, y0, y1; };

__device__ __forceinline__ Rect tile_rect(float cx, float cy, float ex, float ey, int tiles_x,
                                          int tiles_y, int block) {
    Rect r{0, 0, 0, 0};
    if (!(ex > 0.0f) || !(ey > 0.0f)) return r;
    const float b = (float)block;
    float tcx = cx / b, tcy = cy / b, trx = ex / b, try_ = ey / b;
    r.x0 = (int)fminf(fmaxf(tcx - trx, 0.0f), (float)tiles_x);
    r.x1 = (int)fminf(fmaxf(tcx + trx + 1.0f, 0.0f), (float)tiles_x);
    r.y0 = (int)fminf(fmaxf(tcy - try_, 0.0f), (float)tiles_y);
    r.y1 = (int)fminf(fmaxf(tcy + try_ + 1.0f, 0.0f), (float)tiles_y);
    if (r.x1 < r.x0) r.x1 = r.x0;
    if (r.y1 < r.y0) r.y1 = r.y0;
    return r;
}

// Splat -> pixel in affine form.  With the anchored rows (Tu'.z = Tv'.z = 0) the homogeneous point of pixel
// offset d = pixel - anchor is p = k x l, k = d.x Tw - Tu', l = d.y Tw - Tv', which is affine in d:
//   p = d.x A + d.y B + P0,   A = Tv' x Tw,  B = Tw x Tu',  P0 = Tu' x Tv' = (0, 0, Pz)
// (the d.x d.y Tw x Tw term vanishes).  The raster evaluates p this way: 6 products instead of 2 x 3 + 6, and no
// per-pixel cancellation of the d.x d.y terms.
template <typename T> struct AffineHomogT { V3<T> A, B; T Pz; };
template <typename T>
__device__ __forceinline__ AffineHomogT<T> affine_homog(V3<T> Tu, V3<T> Tv, V3<T> Tw) {  // Tu.z = Tv.z = 0 (anchored)
    AffineHomogT<T> a;
    a.A = V3<T>{Tw.z * Tv.y, -(Tw.z * Tv.x), Tw.y * Tv.x - Tw.x * Tv.y};
    a.B = V3<T>{-(Tu.y * Tw.z), Tu.x * Tw.z, Tu.y * Tw.x - Tu.x * Tw.y};
    a.Pz = Tu.x * Tv.y - Tu.y * Tv.x;
    return a;
}
// dL/d(A, B, P0) -> dL/d(Tu', Tv', Tw) (c = a x b: dL/da = b x dL/dc, dL/db = dL/dc x a), including the
// gradients of the z-components of Tu', Tv' (zero-valued, but the anchored vjp holds the anchor fixed)
template <typename T>
__device__ __forceinline__ void affine_homog_vjp(V3<T> Tu, V3<T> Tv, V3<T> Tw, V3<T> dA, V3<T> dB, V3<T> dP0,
                                                 V3<T>& dTu, V3<T>& dTv, V3<T>& dTw) {
    dTu = add3(cross3(dB, Tw), cross3(Tv, dP0));
    dTv = add3(cross3(Tw, dA), cross3(dP0, Tu));
    dTw = add3(cross3(dA, Tv), cross3(Tu, dB));
}

// Raster record layout (GSTEX_REC_FLOATS = 32 floats = 128 B, one cache line), as 8 float4 planes.
enum RecField {
    // dwords [0, 12) (planes 0-2): everything the per-wave cull reads (raster.hip wave_may_hit), so a candidate costs
    // three 16-B loads; every field the photometric backward reads lies in [0, 27) (one contiguous scalar load run
    // per visit)
    R_A = 0, R_B = 3, R_PZ = 6, R_XA = 7, R_YA = 8, R_XY = 9, R_OPAC = 11,
    R_TW = 12, R_RGB = 15, R_TU0 = 18, R_AUU = 19, R_AUV = 20, R_TV0 = 21, R_AVU = 22, R_AVV = 23,
    R_H = 24, R_W = 25, R_OFF = 26, R_NRM = 27,
    R_HM1 = 30, R_WM1 = 31  // (float)(h - 1), (float)(w - 1): exact, the forward's texel clamps without conversions
};
constexpr int kCullPlanes = 3;  // record planes holding the cull fields

// Near-edge-on splats (|normal . view direction| < kHpCos at the splat centre): their homogeneous point p = dx A + dy B +
// (0, 0, Pz) is ill-conditioned in the fp32 record (p.z is a small difference of larger terms), and with it u = p.x / p.z,
// v = p.y / p.z and every means / quats gradient through them.  When the caller passes a row buffer, the
// setup marks such a splat by the sign bit of its record opacity (R_OPAC < 0; every reader takes |R_OPAC|) and writes
// the fp64 values of its affine homography and depth row (HpField) into row g of that buffer; the backward re-evaluates
// dx, dy, p, 1 / p.z, u, v, rho3 and z of those pairs in fp64 (every pair decision stays the fp32 forward's).
#ifndef GSTEX_HP_COS
#define GSTEX_HP_COS 0.1
#endif
constexpr double kHpCos = GSTEX_HP_COS;
enum HpField { H_A = 0, H_B = 3, H_PZ = 6, H_XA = 7, H_YA = 8, H_TW = 9, H_FIELDS = 12 };
static_assert(H_FIELDS == GSTEX_HP_DOUBLES, "gstex_hip.h GSTEX_HP_DOUBLES");

// Screen box of the projected disc u^2 + v^2 <= c2 (compute_aabb with a general cutoff).
// Returns false when the disc reaches the camera plane (unbounded projection).
__device__ __forceinline__ bool ellipse_box(const Homog& h, float c2, float& x0, float& x1, float& y0,
                                            float& y1) {
    const f3 Tu = h.Tu, Tv = h.Tv, Tw = h.Tw;
    const float d = (c2 * (Tw.x * Tw.x) + c2 * (Tw.y * Tw.y)) - Tw.z * Tw.z;
    if (!(d < 0.0f) || !(Tw.z > 0.0f)) return false;
    const float fxy = c2 / d, fz = -1.0f / d;
    const float px = (fxy * (Tu.x * Tw.x) + fxy * (Tu.y * Tw.y)) + fz * (Tu.z * Tw.z);
    const float py = (fxy * (Tv.x * Tw.x) + fxy * (Tv.y * Tw.y)) + fz * (Tv.z * Tw.z);
    const float qx = (fxy * (Tu.x * Tu.x) + fxy * (Tu.y * Tu.y)) + fz * (Tu.z * Tu.z);
    const float qy = (fxy * (Tv.x * Tv.x) + fxy * (Tv.y * Tv.y)) + fz * (Tv.z * Tv.z);
    const float ex = sqrtf(fmaxf(0.0f, px * px - qx)), ey = sqrtf(fmaxf(0.0f, py * py - qy));
    x0 = px - ex; x1 = px + ex; y0 = py - ey; y1 = py + ey;
    return true;
}

// Conservative box of the pixels where a splat can reach alpha >= 1/255: rho <= 2 ln(255 o) for
// rho = u^2 + v^2 (3D disc) or 2 |pix - xy|^2 (2DGS low-pass disc); union of both, +1 px margin.
// Rasterizer waves whose pixel block misses this box skip the splat: an exact cull (the skipped
// pairs would fail the alpha >= 1/255 test anyway).
__device__ __forceinline__ void contribution_box(const Homog& h, float cx, float cy, float opac, float& x0,
                                                 float& x1, float& y0, float& y1) {
    x0 = y0 = 3.0e38f;
    x1 = y1 = -3.0e38f;
    if (!(opac * 255.0f > 1.0f)) return;  // can never pass the alpha test
    const float rm = 2.0f * logf(255.0f * opac) * 1.001f + 1e-3f;
    const float r2 = sqrtf(0.5f * rm);
    float ex0, ex1, ey0, ey1;
    if (!ellipse_box(h, rm, ex0, ex1, ey0, ey1)) {
        x0 = y0 = -3.0e38f;
        x1 = y1 = 3.0e38f;
        return;
    }
    x0 = fminf(ex0, cx - r2) - 1.0f;
    x1 = fmaxf(ex1, cx + r2) + 1.0f;
    y0 = fminf(ey0, cy - r2) - 1.0f;
    y1 = fmaxf(ey1, cy + r2) + 1.0f;
}

// Partial-row layout: dL/d(A, B, P0) of the affine homography, the AA low-pass centre gradient, opacity, colour,
// texture-coordinate affine, and (rows of a backward with depth / normal gradients only) normal and the direct
// dL/dTw of the depth.  A row holds 24 values (flag 1) or, with depth / normal gradients, 32 (flag 2); rows
// are GSTEX_PARTIAL_FLOATS = 32 floats apart.
enum PartField {
    P_A = 0, P_B = 3, P_P0 = 6, P_XY = 9, P_OPAC = 11, P_RGB = 12,
    P_TU0 = 15, P_AUU = 16, P_AUV = 17, P_TV0 = 18, P_AVU = 19, P_AVV = 20, P_NRM = 21, P_TW = 24
};
// Backward unit order (binning.hip gstex_unit_order): counting-sort bins = XCD group x descending cost bucket.
constexpr int kUnitBuckets = 1024;
constexpr int kUnitGroups = 8;
constexpr int kUnitBins = kUnitBuckets * kUnitGroups;
__device__ __forceinline__ int unit_bin(int key) {
    const int c = key & 0xFFFFFF, g = (key >> 24) & (kUnitGroups - 1);
    return g * kUnitBuckets + (kUnitBuckets - 1 - min(c, kUnitBuckets - 1));
}
// Internal entry (binning.hip) for the raster backward: the order from a histogram the forward already built in
// scratch[0, kUnitBins) (scratch[kUnitBins, 2 kUnitBins) zeroed with it: the placement counters); order[] entries are
// unit + 1 (0 = no unit at that launch position; the caller zeroed it).
int unit_order_from_hist(int32_t n_units, const int32_t* unit_key, int32_t* unit_order, int32_t* scratch,
                         hipStream_t st);

constexpr int kPartRow = 24;     // values per row without geometry gradients
constexpr int kPartRowGeo = 32;  // with (27 used)

// Bilinear lookup into one splat's h x w texel block (corner-aligned: texel (i,j) sits at uv
// (i/h, j/w), matching texture_dims_to_query, jagged_texture.py:23-34; clamp to edge).
struct Bilerp { int i0, i1, j0, j1; float ax, ay; bool in_u, in_v; };

// From the sample point in texel units (xr, yr) = (tu h, tv w); hm1, wm1 = (float)(h - 1), (float)(w - 1) (exact).
// The clamps to [0, h - 1] are single v_med3_f32 (= fminf(fmaxf(x, 0), h - 1) for every non-NaN x).
__device__ __forceinline__ Bilerp bilerp_xy(float xr, float yr, int h, int w, float hm1, float wm1) {
    Bilerp b;
    float x = __builtin_amdgcn_fmed3f(xr, 0.0f, hm1);
    float y = __builtin_amdgcn_fmed3f(yr, 0.0f, wm1);
    b.in_u = (xr > 0.0f) && (xr < hm1);
    b.in_v = (yr > 0.0f) && (yr < wm1);
    b.i0 = (int)x; b.j0 = (int)y;
    b.i1 = min(b.i0 + 1, h - 1);
    b.j1 = min(b.j0 + 1, w - 1);
    // x, y >= 0: x - floor(x) is exact and < 1, so v_fract_f32 (S0 - floor(S0)) gives x - (float)i0 bit for bit
    b.ax = __builtin_amdgcn_fractf(x);
    b.ay = __builtin_amdgcn_fractf(y);
    return b;
}

__device__ __forceinline__ Bilerp bilerp_coords(float tu, float tv, int h, int w) {
    const float hf = (float)h, wf = (float)w;
    return bilerp_xy(tu * hf, tv * wf, h, w, hf - 1.0f, wf - 1.0f);
}

__device__ __forceinline__ float bilerp_mix(float v00, float v01, float v10, float v11, float ax,
                                            float ay) {
    float top = (1.0f - ay) * v00 + ay * v01;
    float bot = (1.0f - ay) * v10 + ay * v11;
    return (1.0f - ax) * top + ax * bot;
}


}  // namespace gstex
