// loss.hip — the GStex photometric loss, fused: background composite, clamp, 0.8 L1 + 0.2 (1 - SSIM).
//
//   gstex_loss_fwd / gstex_loss_bwd  <- gstex.py:1204-1205 (rgb = clamp(img + tex + (1-alpha) bg))
//                                       and gstex.py:1301-1322 (0.8 * L1 + 0.2 * (1 - SSIM)),
//                                       SSIM with pytorch_msssim semantics (gstex.py:351): 11-tap
//                                       gaussian window (sigma 1.5, weights supplied by the caller),
//                                       VALID filtering, C1 = 0.01^2, C2 = 0.03^2, mean over the map.
//     X = gt, Y = rgb; only Y is differentiated.
//
// Forward, one 16x16 workgroup tile per image block and channel: the 26x26 input window is
// staged in LDS, filtered separably (rows, then columns) into mu1, mu2, E[X^2], E[Y^2], E[XY];
// every valid position p writes s(p) into a per-workgroup partial sum and the three partials the
// backward needs, dS/d mu2, dS/d E[Y^2], dS/d E[XY] (gmaps).  A one-workgroup kernel then reduces
// the partial sums in a fixed order (deterministic loss).
// Backward: dS/dY(q) = sum over the windows containing q of w * (G_mu2 + 2 Y(q) G_yy + X(q) G_xy),
// the transposed separable filter of the gmaps, evaluated the same tiled way, channel by channel; the
// composite's backward (d_img, d_tex, d_alpha) is written by the same workgroup once a pixel's three channels are
// done (no dL/drgb buffer, no separate scatter launch).
#include "gstex_common.h"
#include "gstex_error.h"

namespace {

constexpr int kLT = 16;            // output tile side
constexpr int kWin = 11;           // gaussian window
constexpr int kHalo = kWin - 1;    // 10
constexpr int kReg = kLT + kHalo;  // 26: staged window side
constexpr float kC1 = 0.01f * 0.01f;
constexpr float kC2 = 0.03f * 0.03f;

struct Win {
    float w[kWin];
};

// rgb = clamp((img + tex) + (1 - alpha) * bg, 0, 1) exactly as gstex.py:1204 evaluates it; `pre`
// returns the unclamped value (the clamp's gradient mask).
__device__ __forceinline__ float composite(const float* img, const float* tex, const float* alpha, const float* bg,
                                           int C, size_t pix, int c, float& pre) {
    const float v = (img[3 * pix + c] + tex[(size_t)C * pix + c]) + (1.0f - alpha[pix]) * bg[c];
    pre = v;
    return fminf(fmaxf(v, 0.0f), 1.0f);
}

#ifndef GSTEX_LOSS_XCD
#define GSTEX_LOSS_XCD 1
#endif
// XCD-aware tile order: workgroups are dispatched round-robin over the 8 XCDs, each with its own L2, so
// in launch order neighbouring tiles (which share their 10-pixel halos) land on different XCDs and the
// halos come from HBM again.  Launch slot L goes to XCD L % 8; giving XCD x the contiguous run of tiles
// [x * n/8, ...) in (bx, by, c) order keeps neighbours on one L2.  A bijection of the launch slots.
struct LossTile {
    int bx, by, c;
};
__device__ __forceinline__ LossTile loss_tile() {
    if (!GSTEX_LOSS_XCD) return LossTile{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
    const int gx = gridDim.x, gy = gridDim.y;
    const int n = gx * gy * gridDim.z;
    const int L = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int per = n / 8, rem = n % 8, xcd = L % 8;
    const int t = xcd * per + min(xcd, rem) + L / 8;
    return LossTile{t % gx, (t / gx) % gy, t / (gx * gy)};
}

__global__ __launch_bounds__(256) void loss_fwd_kernel(int H, int W, int C, const float* __restrict__ img,
                                                       const float* __restrict__ tex,
                                                       const float* __restrict__ alpha,
                                                       const float* __restrict__ bg, const float* __restrict__ gt,
                                                       Win win, float* __restrict__ rgb_out,
                                                       float* __restrict__ gmaps, float2* __restrict__ part) {
    __shared__ float s_x[kReg][kReg + 1], s_y[kReg][kReg + 1];
    __shared__ float s_h[5][kReg][kLT + 1];
    __shared__ float s_red[2][8];
    const LossTile lt = loss_tile();
    const int c = lt.c;
    const int x0 = lt.bx * kLT, y0 = lt.by * kLT;
    const int tid = threadIdx.x;
    const int Hv = H - kHalo, Wv = W - kHalo;
    float l1 = 0.f;
    for (int i = tid; i < kReg * kReg; i += 256) {
        const int ry = i / kReg, rx = i % kReg;
        const int y = y0 + ry, x = x0 + rx;
        float xv = 0.f, yv = 0.f;
        if (y < H && x < W) {
            const size_t pix = (size_t)y * W + x;
            float pre;
            yv = composite(img, tex, alpha, bg, C, pix, c, pre);
            xv = gt[3 * pix + c];
            if (rx < kLT && ry < kLT) {  // each pixel's L1 term and rgb belong to the tile whose core holds it
                l1 += fabsf(xv - yv);
                if (rgb_out) rgb_out[3 * pix + c] = yv;
            }
        }
        s_x[ry][rx] = xv;
        s_y[ry][rx] = yv;
    }
    __syncthreads();
    // rows: 26 x 16 horizontal filters of the five quantities (fused multiply-adds: the window sums need no fixed
    // operation order -- the loss and its gradient are compared with tolerances, only the composite bit for bit)
    for (int i = tid; i < kReg * kLT; i += 256) {
#pragma clang fp contract(fast)
        const int ry = i / kLT, cx = i % kLT;
        float a = 0.f, b = 0.f, aa = 0.f, bb = 0.f, ab = 0.f;
#pragma unroll
        for (int k = 0; k < kWin; ++k) {
            const float xv = s_x[ry][cx + k], yv = s_y[ry][cx + k];
            a += win.w[k] * xv;
            b += win.w[k] * yv;
            aa += win.w[k] * (xv * xv);
            bb += win.w[k] * (yv * yv);
            ab += win.w[k] * (xv * yv);
        }
        s_h[0][ry][cx] = a;
        s_h[1][ry][cx] = b;
        s_h[2][ry][cx] = aa;
        s_h[3][ry][cx] = bb;
        s_h[4][ry][cx] = ab;
    }
    __syncthreads();
    // columns + the SSIM map at this thread's position
    const int cy = tid >> 4, cx = tid & 15;
    const int py = y0 + cy, px = x0 + cx;
    float ssum = 0.f;
    if (py < Hv && px < Wv) {
#pragma clang fp contract(fast)
        float q[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < kWin; ++k)
#pragma unroll
            for (int m = 0; m < 5; ++m) q[m] += win.w[k] * s_h[m][cy + k][cx];
        const float mu1 = q[0], mu2 = q[1];
        const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
        const float s11 = q[2] - mu1_sq, s22 = q[3] - mu2_sq, s12 = q[4] - mu1_mu2;
        const float A = 2.0f * mu1_mu2 + kC1, B = 2.0f * s12 + kC2;
        const float Cc = mu1_sq + mu2_sq + kC1, D = s11 + s22 + kC2;
        const float cs = B / D;
        const float s = (A / Cc) * cs;
        ssum = s;
        // dS/d mu2 (through mu2, sigma2^2 = E[Y^2] - mu2^2, sigma12 = E[XY] - mu1 mu2), dS/dE[Y^2], dS/dE[XY]
        const float ds_dmu2 = s * (2.0f * mu1 / A - 2.0f * mu2 / Cc);
        const float ds_ds22 = -s / D;
        const float ds_ds12 = 2.0f * s / B;
        const size_t o = ((size_t)c * Hv + py) * Wv + px;
        const size_t plane = (size_t)3 * Hv * Wv;
        gmaps[o] = ds_dmu2 - 2.0f * mu2 * ds_ds22 - mu1 * ds_ds12;
        gmaps[plane + o] = ds_ds22;
        gmaps[2 * plane + o] = ds_ds12;
    }
    // workgroup sums (fixed order: wave reduce, then the 4 waves in order)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        ssum += __shfl_xor(ssum, off, 64);
        l1 += __shfl_xor(l1, off, 64);
    }
    if ((tid & 63) == 0) {
        s_red[0][tid >> 6] = ssum;
        s_red[1][tid >> 6] = l1;
    }
    __syncthreads();
    if (tid == 0) {
        const int b = (lt.c * gridDim.y + lt.by) * gridDim.x + lt.bx;  // tile index: fixed reduction order
        part[b] = make_float2(((s_red[0][0] + s_red[0][1]) + s_red[0][2]) + s_red[0][3],
                              ((s_red[1][0] + s_red[1][1]) + s_red[1][2]) + s_red[1][3]);
    }
}

__global__ __launch_bounds__(1024) void loss_reduce_kernel(int nparts, const float2* __restrict__ part, double inv_n1,
                                                           double inv_np, float w_l1, float w_ssim,
                                                           float* __restrict__ loss) {
    __shared__ double s_s[1024], s_l[1024];
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < nparts; i += 1024) {
        a += (double)part[i].x;
        b += (double)part[i].y;
    }
    s_s[threadIdx.x] = a;
    s_l[threadIdx.x] = b;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            s_s[threadIdx.x] += s_s[threadIdx.x + o];
            s_l[threadIdx.x] += s_l[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float l1 = (float)(s_l[0] * inv_n1);
        const float ssim = (float)(s_s[0] * inv_np);
        loss[0] = w_l1 * l1 + w_ssim * (1.0f - ssim);
        loss[1] = l1;
        loss[2] = ssim;
    }
}

__global__ __launch_bounds__(256) void loss_bwd_kernel(int H, int W, int C, const float* __restrict__ img,
                                                       const float* __restrict__ tex,
                                                       const float* __restrict__ alpha,
                                                       const float* __restrict__ bg, const float* __restrict__ gt,
                                                       Win win, const float* __restrict__ gmaps,
                                                       const float* __restrict__ grad_loss, float k_l1,
                                                       float k_ssim, float* __restrict__ d_img,
                                                       float* __restrict__ d_tex, float* __restrict__ d_alpha) {
    // one workgroup per 16x16 tile, the three channels in turn; the composite's backward (d_img, d_tex, d_alpha)
    // written at the end, once every channel's dL/drgb of the pixel is known
    __shared__ float s_g[3][kReg][kReg + 1];
    __shared__ float s_h[3][kReg][kLT + 1];
    const LossTile lt = loss_tile();
    const int x0 = lt.bx * kLT, y0 = lt.by * kLT;  // output pixels [x0, x0+16)
    const int tid = threadIdx.x;
    const int Hv = H - kHalo, Wv = W - kHalo;
    const size_t plane = (size_t)3 * Hv * Wv;
    const int cy = tid >> 4, cx = tid & 15;
    const int qy = y0 + cy, qx = x0 + cx;
    const bool out = qy < H && qx < W;
    const size_t pix = (size_t)qy * W + qx;
    const float gl = grad_loss[0];
    float gch[3];
    for (int c = 0; c < 3; ++c) {
        if (c > 0) __syncthreads();  // the previous channel's passes are done with s_g / s_h
        // gmaps over positions [x0 - 10, x0 + 16)
        for (int i = tid; i < kReg * kReg; i += 256) {
            const int ry = i / kReg, rx = i % kReg;
            const int gy = y0 - kHalo + ry, gx = x0 - kHalo + rx;
            float g0 = 0.f, g1 = 0.f, g2 = 0.f;
            if (gy >= 0 && gx >= 0 && gy < Hv && gx < Wv) {
                const size_t o = ((size_t)c * Hv + gy) * Wv + gx;
                g0 = gmaps[o];
                g1 = gmaps[plane + o];
                g2 = gmaps[2 * plane + o];
            }
            s_g[0][ry][rx] = g0;
            s_g[1][ry][rx] = g1;
            s_g[2][ry][rx] = g2;
        }
        __syncthreads();
        // transposed rows: for output column hx, sum_k w[k] G(position hx + 10 - k)
        for (int i = tid; i < kReg * kLT; i += 256) {
#pragma clang fp contract(fast)
            const int ry = i / kLT, hx = i % kLT;
            float a = 0.f, b = 0.f, d = 0.f;
#pragma unroll
            for (int k = 0; k < kWin; ++k) {
                a += win.w[k] * s_g[0][ry][hx + kHalo - k];
                b += win.w[k] * s_g[1][ry][hx + kHalo - k];
                d += win.w[k] * s_g[2][ry][hx + kHalo - k];
            }
            s_h[0][ry][hx] = a;
            s_h[1][ry][hx] = b;
            s_h[2][ry][hx] = d;
        }
        __syncthreads();
        gch[c] = 0.f;
        if (out) {
#pragma clang fp contract(fast)
            float t0 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
            for (int k = 0; k < kWin; ++k) {
                t0 += win.w[k] * s_h[0][cy + kHalo - k][cx];
                t1 += win.w[k] * s_h[1][cy + kHalo - k][cx];
                t2 += win.w[k] * s_h[2][cy + kHalo - k][cx];
            }
            float pre;
            const float yv = composite(img, tex, alpha, bg, C, pix, c, pre);
            const float xv = gt[3 * pix + c];
            const float dS = (t0 + 2.0f * yv * t1) + xv * t2;
            const float diff = xv - yv;
            const float sgn = diff > 0.f ? 1.0f : (diff < 0.f ? -1.0f : 0.0f);
            // L = w1 * mean|X - Y| + w2 * (1 - mean s): dL/dY = -w1 sign(X - Y) / N1 - w2 dS / Np
            float g = -(k_l1 * sgn) - k_ssim * dS;
            g *= gl;
            gch[c] = (pre >= 0.0f && pre <= 1.0f) ? g : 0.0f;
        }
    }
    if (!out) return;
    // rgb = clamp((img + tex) + (1 - alpha) bg): d_img = d_tex[0..2] = dL/drgb, channels >= 3 get zero,
    // d_alpha = -sum_c dL/drgb_c bg_c
    d_img[3 * pix] = gch[0];
    d_img[3 * pix + 1] = gch[1];
    d_img[3 * pix + 2] = gch[2];
    for (int c = 0; c < C; ++c) d_tex[(size_t)C * pix + c] = c == 0 ? gch[0] : (c == 1 ? gch[1] : (c == 2 ? gch[2] : 0.0f));
    d_alpha[pix] = -((gch[0] * bg[0] + gch[1] * bg[1]) + gch[2] * bg[2]);
}

}  // namespace

using namespace gstex;

// forward: one workgroup per (tile, channel); backward: one per tile (its three channels in turn)
static int loss_grid(int H, int W, dim3& grid, int channels = 3) {
    grid = dim3((unsigned)((W + kLT - 1) / kLT), (unsigned)((H + kLT - 1) / kLT), (unsigned)channels);
    return (int)(grid.x * grid.y * grid.z);
}

extern "C" size_t gstex_loss_workspace_size(int32_t H, int32_t W) {
    if (H <= kHalo || W <= kHalo) return 0;
    dim3 g;
    const size_t parts = (size_t)loss_grid(H, W, g) * sizeof(float2);
    const size_t gm = (size_t)3 * 3 * (H - kHalo) * (W - kHalo) * sizeof(float);
    return ((parts + 255) & ~(size_t)255) + gm;
}

static void loss_ws(int H, int W, void* ws, float2** part, float** gmaps) {
    dim3 g;
    const size_t parts = (size_t)loss_grid(H, W, g) * sizeof(float2);
    char* b = (char*)ws;
    *part = (float2*)b;
    b += (parts + 255) & ~(size_t)255;
    *gmaps = (float*)b;
}

extern "C" int gstex_loss_fwd(int32_t H, int32_t W, int32_t C, const float* img, const float* tex,
                              const float* alpha, const float* background, const float* gt, const float* window,
                              float ssim_lambda, float* rgb_out, float* loss_out, void* workspace,
                              size_t workspace_bytes, void* stream) {
    GSTEX_REQUIRE(H > kHalo && W > kHalo, "gstex_loss_fwd: image must be larger than the %d-tap window (%dx%d)",
                  kWin, H, W);
    GSTEX_REQUIRE(C >= 3 && C <= 8, "gstex_loss_fwd: tex channels must be in [3, 8] (got %d)", C);
    GSTEX_REQUIRE(img && tex && alpha && background && gt && window && loss_out, "gstex_loss_fwd: null pointer");
    GSTEX_REQUIRE(workspace && workspace_bytes >= gstex_loss_workspace_size(H, W),
                  "gstex_loss_fwd: workspace too small");
    Win win;
    for (int k = 0; k < kWin; ++k) win.w[k] = window[k];  // host array
    float2* part;
    float* gmaps;
    loss_ws(H, W, workspace, &part, &gmaps);
    dim3 grid;
    const int nparts = loss_grid(H, W, grid);
    hipStream_t st = as_stream(stream);
    loss_fwd_kernel<<<grid, 256, 0, st>>>(H, W, C, img, tex, alpha, background, gt, win, rgb_out, gmaps, part);
    loss_reduce_kernel<<<1, 1024, 0, st>>>(nparts, part, 1.0 / (3.0 * H * W), 1.0 / (3.0 * (H - kHalo) * (W - kHalo)),
                                           1.0f - ssim_lambda, ssim_lambda, loss_out);
    return launch_status("gstex_loss_fwd");
}

extern "C" int gstex_loss_bwd(int32_t H, int32_t W, int32_t C, const float* img, const float* tex,
                              const float* alpha, const float* background, const float* gt, const float* window,
                              float ssim_lambda, const float* grad_loss, float* d_img, float* d_tex, float* d_alpha,
                              void* workspace, size_t workspace_bytes, void* stream) {
    GSTEX_REQUIRE(H > kHalo && W > kHalo, "gstex_loss_bwd: image must be larger than the %d-tap window", kWin);
    GSTEX_REQUIRE(C >= 3 && C <= 8, "gstex_loss_bwd: tex channels must be in [3, 8] (got %d)", C);
    GSTEX_REQUIRE(img && tex && alpha && background && gt && window && grad_loss && d_img && d_tex && d_alpha,
                  "gstex_loss_bwd: null pointer");
    GSTEX_REQUIRE(workspace && workspace_bytes >= gstex_loss_workspace_size(H, W),
                  "gstex_loss_bwd: workspace too small");
    Win win;
    for (int k = 0; k < kWin; ++k) win.w[k] = window[k];
    float2* part;
    float* gmaps;
    loss_ws(H, W, workspace, &part, &gmaps);
    dim3 grid;
    loss_grid(H, W, grid, 1);
    hipStream_t st = as_stream(stream);
    const float k_l1 = (float)((1.0 - ssim_lambda) / (3.0 * H * W));
    const float k_ssim = (float)(ssim_lambda / (3.0 * (H - kHalo) * (W - kHalo)));
    loss_bwd_kernel<<<grid, 256, 0, st>>>(H, W, C, img, tex, alpha, background, gt, win, gmaps, grad_loss, k_l1,
                                          k_ssim, d_img, d_tex, d_alpha);
    return launch_status("gstex_loss_bwd");
}
