// sh_texture.hip — spherical-harmonics colour and jagged-texture resampling.
//
//   gstex_sh_fwd / gstex_sh_bwd      <- gstex_cuda.sh.spherical_harmonics (gstex.py:1109,1111;
//                                       exporter.py:40).  Real SH basis of the gsplat-0.1 lineage,
//                                       degree <= 4, result WITHOUT the +0.5 offset (the caller
//                                       zeroes the DC term, gstex.py:1100).  Gradient w.r.t. the
//                                       coefficients only (the caller detaches viewdirs).
//   gstex_texture_sample(_bwd)       <- gstex_cuda.texture_sample.texture_sample
//                                       (models/jagged_texture.py:138): bilinear resample of each
//                                       splat's old texel block at new texel-centre UVs, with the
//                                       same sampler the rasterizer uses (gstex_common.h).
#include "gstex_common.h"
#include "gstex_error.h"
#include "splat_math.h"  // sh_basis, sh_colour

using namespace gstex;

namespace {

// coeffs[i][k - k0] holds basis k (k0 = 1: the DC coefficient is implicitly zero, gstex.py:1100 zeroes it;
// starting the sum at +0 without the zero DC product gives the same bits as with it)
__global__ __launch_bounds__(256) void sh_fwd_kernel(int n, int degree, int k0, int K, const float* __restrict__ dirs,
                                                     const float* __restrict__ coeffs, float* __restrict__ out) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float b[25];
    sh_basis(degree, dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2], b);
    const int nb = (degree + 1) * (degree + 1);
    const float* c = coeffs + (size_t)i * K * 3 - 3 * k0;
    float r0 = 0.f, r1 = 0.f, r2 = 0.f;
    for (int k = k0; k < nb; ++k) {
        r0 = r0 + b[k] * c[3 * k];
        r1 = r1 + b[k] * c[3 * k + 1];
        r2 = r2 + b[k] * c[3 * k + 2];
    }
    out[3 * i] = r0;
    out[3 * i + 1] = r1;
    out[3 * i + 2] = r2;
}

__global__ __launch_bounds__(256) void sh_bwd_kernel(int n, int degree, int k0, int K, const float* __restrict__ dirs,
                                                     const float* __restrict__ v_out, float* __restrict__ v_coeffs) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    sh_grad_row(degree, k0, K, dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2], v_out[3 * i], v_out[3 * i + 1],
                v_out[3 * i + 2], v_coeffs + (size_t)i * K * 3);
}

// The same two kernels with the coefficient rows staged through LDS: a workgroup's 128 splats own one
// contiguous span of coefficients, read (forward) or written (backward) with consecutive lanes on
// consecutive words; the per-thread strided rows (180 B apart at K = 15) made every load instruction
// touch 64 cache lines.  Same arithmetic and order as above.  Used for K <= kShStagedMaxK.  The span is
// copied whole (rows of 3K words, also when the degree uses fewer) as 16-B vectors, several in flight per
// thread, when it is 16-B aligned (the scalar copy with a division per word was the kernels' latency chain).
constexpr int kShBlock = 128;
constexpr int kShStagedMaxK = 25;

__global__ __launch_bounds__(kShBlock) void sh_fwd_staged_kernel(int n, int degree, int k0, int K,
                                                                const float* __restrict__ dirs,
                                                                const float* __restrict__ coeffs,
                                                                float* __restrict__ out) {
    extern __shared__ float s_c[];
    const int t = threadIdx.x;
    const int i0 = blockIdx.x * kShBlock;
    const int cnt = min(kShBlock, n - i0);
    const int kw = K * 3;  // words per splat row
    sh_copy_span<kShBlock>(s_c, coeffs + (size_t)i0 * kw, cnt * kw);
    __syncthreads();
    if (t >= cnt) return;
    const int i = i0 + t;
    float r0, r1, r2;
    sh_colour(degree, k0, dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2], s_c + t * kw - 3 * k0, r0, r1, r2);
    out[3 * i] = r0;
    out[3 * i + 1] = r1;
    out[3 * i + 2] = r2;
}

__global__ __launch_bounds__(kShBlock) void sh_bwd_staged_kernel(int n, int degree, int k0, int K,
                                                                const float* __restrict__ dirs,
                                                                const float* __restrict__ v_out,
                                                                float* __restrict__ v_coeffs) {
    extern __shared__ float s_c[];
    const int t = threadIdx.x;
    const int i0 = blockIdx.x * kShBlock;
    const int cnt = min(kShBlock, n - i0);
    const int kw = K * 3;
    if (t < cnt) {
        const int i = i0 + t;
        sh_grad_row(degree, k0, K, dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2], v_out[3 * i], v_out[3 * i + 1],
                    v_out[3 * i + 2], s_c + t * kw);
    }
    __syncthreads();
    sh_copy_span<kShBlock>(v_coeffs + (size_t)i0 * kw, s_c, cnt * kw);
}

// One thread per (query, channel-group): query q reads its 4 corner texels.
__global__ __launch_bounds__(256) void texture_sample_kernel(long long nq, int C, const int32_t* __restrict__ qd,
                                                             const float* __restrict__ tex,
                                                             const float* __restrict__ uv, float* __restrict__ out) {
    long long q = (long long)blockIdx.x * 256 + threadIdx.x;
    if (q >= nq) return;
    const int h = qd[3 * q], w = qd[3 * q + 1], off = qd[3 * q + 2];
    float* o = out + q * C;
    if (h * w <= 0) {
        for (int c = 0; c < C; ++c) o[c] = 0.0f;
        return;
    }
    const Bilerp b = bilerp_coords(uv[2 * q], uv[2 * q + 1], h, w);
    const size_t o00 = (size_t)(off + b.i0 * w + b.j0) * C, o01 = (size_t)(off + b.i0 * w + b.j1) * C;
    const size_t o10 = (size_t)(off + b.i1 * w + b.j0) * C, o11 = (size_t)(off + b.i1 * w + b.j1) * C;
    for (int c = 0; c < C; ++c) o[c] = bilerp_mix(tex[o00 + c], tex[o01 + c], tex[o10 + c], tex[o11 + c], b.ax, b.ay);
}

__global__ __launch_bounds__(256) void texture_sample_bwd_kernel(long long nq, int C, const int32_t* __restrict__ qd,
                                                                 const float* __restrict__ uv,
                                                                 const float* __restrict__ v_out,
                                                                 float* __restrict__ v_tex) {
    long long q = (long long)blockIdx.x * 256 + threadIdx.x;
    if (q >= nq) return;
    const int h = qd[3 * q], w = qd[3 * q + 1], off = qd[3 * q + 2];
    if (h * w <= 0) return;
    const Bilerp b = bilerp_coords(uv[2 * q], uv[2 * q + 1], h, w);
    const size_t o00 = (size_t)(off + b.i0 * w + b.j0) * C, o01 = (size_t)(off + b.i0 * w + b.j1) * C;
    const size_t o10 = (size_t)(off + b.i1 * w + b.j0) * C, o11 = (size_t)(off + b.i1 * w + b.j1) * C;
    const float w00 = (1.0f - b.ax) * (1.0f - b.ay), w01 = (1.0f - b.ax) * b.ay;
    const float w10 = b.ax * (1.0f - b.ay), w11 = b.ax * b.ay;
    for (int c = 0; c < C; ++c) {
        const float g = v_out[q * C + c];
        atomicAdd(v_tex + o00 + c, g * w00);
        atomicAdd(v_tex + o01 + c, g * w01);
        atomicAdd(v_tex + o10 + c, g * w10);
        atomicAdd(v_tex + o11 + c, g * w11);
    }
}

}  // namespace

extern "C" int gstex_sh_fwd(int32_t n, int32_t degree, int32_t n_coeffs, const float* viewdirs, const float* coeffs,
                            float* colors, void* stream) {
    GSTEX_REQUIRE(n >= 0 && degree >= 0 && degree <= 4, "gstex_sh_fwd: degree must be in [0, 4] (got %d)", degree);
    GSTEX_REQUIRE(n_coeffs >= (degree + 1) * (degree + 1), "gstex_sh_fwd: %d coefficients < (degree+1)^2 = %d",
                  n_coeffs, (degree + 1) * (degree + 1));
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(viewdirs && coeffs && colors, "gstex_sh_fwd: null pointer");
    if (n_coeffs <= kShStagedMaxK)
        sh_fwd_staged_kernel<<<div_up(n, kShBlock), kShBlock, (size_t)kShBlock * n_coeffs * 3 * sizeof(float),
                               as_stream(stream)>>>(n, degree, 0, n_coeffs, viewdirs, coeffs, colors);
    else
        sh_fwd_kernel<<<div_up(n, 256), 256, 0, as_stream(stream)>>>(n, degree, 0, n_coeffs, viewdirs, coeffs, colors);
    return launch_status("gstex_sh_fwd");
}

extern "C" int gstex_sh_bwd(int32_t n, int32_t degree, int32_t n_coeffs, const float* viewdirs,
                            const float* v_colors, float* v_coeffs, void* stream) {
    GSTEX_REQUIRE(n >= 0 && degree >= 0 && degree <= 4, "gstex_sh_bwd: degree must be in [0, 4]");
    GSTEX_REQUIRE(n_coeffs >= (degree + 1) * (degree + 1), "gstex_sh_bwd: too few coefficients");
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(viewdirs && v_colors && v_coeffs, "gstex_sh_bwd: null pointer");
    if (n_coeffs <= kShStagedMaxK)
        sh_bwd_staged_kernel<<<div_up(n, kShBlock), kShBlock, (size_t)kShBlock * n_coeffs * 3 * sizeof(float),
                               as_stream(stream)>>>(n, degree, 0, n_coeffs, viewdirs, v_colors, v_coeffs);
    else
        sh_bwd_kernel<<<div_up(n, 256), 256, 0, as_stream(stream)>>>(n, degree, 0, n_coeffs, viewdirs, v_colors, v_coeffs);
    return launch_status("gstex_sh_bwd");
}

extern "C" int gstex_sh_rest_fwd(int32_t n, int32_t degree, int32_t n_rest, const float* viewdirs,
                                 const float* coeffs_rest, float* colors, void* stream) {
    GSTEX_REQUIRE(n >= 0 && degree >= 0 && degree <= 4, "gstex_sh_rest_fwd: degree must be in [0, 4] (got %d)", degree);
    GSTEX_REQUIRE(n_rest >= (degree + 1) * (degree + 1) - 1, "gstex_sh_rest_fwd: %d coefficients < (degree+1)^2 - 1",
                  n_rest);
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(viewdirs && colors && (coeffs_rest || n_rest == 0), "gstex_sh_rest_fwd: null pointer");
    if (n_rest <= kShStagedMaxK)
        sh_fwd_staged_kernel<<<div_up(n, kShBlock), kShBlock, (size_t)kShBlock * n_rest * 3 * sizeof(float),
                               as_stream(stream)>>>(n, degree, 1, n_rest, viewdirs, coeffs_rest, colors);
    else
        sh_fwd_kernel<<<div_up(n, 256), 256, 0, as_stream(stream)>>>(n, degree, 1, n_rest, viewdirs, coeffs_rest, colors);
    return launch_status("gstex_sh_rest_fwd");
}

extern "C" int gstex_sh_rest_bwd(int32_t n, int32_t degree, int32_t n_rest, const float* viewdirs,
                                 const float* v_colors, float* v_coeffs_rest, void* stream) {
    GSTEX_REQUIRE(n >= 0 && degree >= 0 && degree <= 4, "gstex_sh_rest_bwd: degree must be in [0, 4]");
    GSTEX_REQUIRE(n_rest >= 0, "gstex_sh_rest_bwd: n_rest < 0");
    if (n == 0 || n_rest == 0) return GSTEX_OK;
    GSTEX_REQUIRE(viewdirs && v_colors && v_coeffs_rest, "gstex_sh_rest_bwd: null pointer");
    if (n_rest <= kShStagedMaxK)
        sh_bwd_staged_kernel<<<div_up(n, kShBlock), kShBlock, (size_t)kShBlock * n_rest * 3 * sizeof(float),
                               as_stream(stream)>>>(n, degree, 1, n_rest, viewdirs, v_colors, v_coeffs_rest);
    else
        sh_bwd_kernel<<<div_up(n, 256), 256, 0, as_stream(stream)>>>(n, degree, 1, n_rest, viewdirs, v_colors, v_coeffs_rest);
    return launch_status("gstex_sh_rest_bwd");
}

extern "C" int gstex_texture_sample(int64_t n_query, int32_t channels, const int32_t* query_dims,
                                    const float* texture, int64_t n_texels, const float* uv, float* out,
                                    void* stream) {
    (void)n_texels;
    GSTEX_REQUIRE(n_query >= 0 && channels >= 1, "gstex_texture_sample: invalid arguments");
    if (n_query == 0) return GSTEX_OK;
    GSTEX_REQUIRE(query_dims && uv && out, "gstex_texture_sample: null pointer");
    texture_sample_kernel<<<div_up(n_query, 256), 256, 0, as_stream(stream)>>>(n_query, channels, query_dims, texture,
                                                                               uv, out);
    return launch_status("gstex_texture_sample");
}

extern "C" int gstex_texture_sample_bwd(int64_t n_query, int32_t channels, const int32_t* query_dims,
                                        int64_t n_texels, const float* uv, const float* v_out, float* v_texture,
                                        void* stream) {
    (void)n_texels;
    GSTEX_REQUIRE(n_query >= 0 && channels >= 1, "gstex_texture_sample_bwd: invalid arguments");
    if (n_query == 0) return GSTEX_OK;
    GSTEX_REQUIRE(query_dims && uv && v_out && v_texture, "gstex_texture_sample_bwd: null pointer");
    texture_sample_bwd_kernel<<<div_up(n_query, 256), 256, 0, as_stream(stream)>>>(n_query, channels, query_dims, uv,
                                                                                   v_out, v_texture);
    return launch_status("gstex_texture_sample_bwd");
}
