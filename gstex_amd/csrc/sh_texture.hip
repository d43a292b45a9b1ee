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

using namespace gstex;

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
    float b[25];
    sh_basis(degree, dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2], b);
    const int nb = (degree + 1) * (degree + 1);
    const float g0 = v_out[3 * i], g1 = v_out[3 * i + 1], g2 = v_out[3 * i + 2];
    float* vc = v_coeffs + (size_t)i * K * 3;
    for (int k = 0; k < K; ++k) {
        const float bk = (k + k0 < nb) ? b[k + k0] : 0.0f;
        vc[3 * k] = bk * g0;
        vc[3 * k + 1] = bk * g1;
        vc[3 * k + 2] = bk * g2;
    }
}

// The same two kernels with the coefficient rows staged through LDS: a workgroup's 128 splats own one
// contiguous span of coefficients, read (forward) or written (backward) with consecutive lanes on
// consecutive words; the per-thread strided rows (180 B apart at K = 15) made every load instruction
// touch 64 cache lines.  Same arithmetic and order as above.  Used for K <= kShStagedMaxK.  The span is
// copied whole (rows of 3K words, also when the degree uses fewer) as 16-B vectors, several in flight per
// thread, when it is 16-B aligned (the scalar copy with a division per word was the kernels' latency chain).
constexpr int kShBlock = 128;
constexpr int kShStagedMaxK = 25;
__device__ __forceinline__ void sh_copy_span(float* __restrict__ dst, const float* __restrict__ src, int total) {
    const int t = threadIdx.x;
    int done = 0;
    if ((((uintptr_t)src | (uintptr_t)dst) & 15u) == 0) {
        const int n4 = total >> 2;
        const float4* s4 = reinterpret_cast<const float4*>(src);
        float4* d4 = reinterpret_cast<float4*>(dst);
#pragma unroll 4
        for (int q = t; q < n4; q += kShBlock) d4[q] = s4[q];
        done = n4 << 2;
    }
    for (int q = done + t; q < total; q += kShBlock) dst[q] = src[q];
}

__global__ __launch_bounds__(kShBlock) void sh_fwd_staged_kernel(int n, int degree, int k0, int K,
                                                                const float* __restrict__ dirs,
                                                                const float* __restrict__ coeffs,
                                                                float* __restrict__ out) {
    extern __shared__ float s_c[];
    const int t = threadIdx.x;
    const int i0 = blockIdx.x * kShBlock;
    const int cnt = min(kShBlock, n - i0);
    const int nb = (degree + 1) * (degree + 1);
    const int kw = K * 3;  // words per splat row
    sh_copy_span(s_c, coeffs + (size_t)i0 * kw, cnt * kw);
    __syncthreads();
    if (t >= cnt) return;
    const int i = i0 + t;
    float b[25];
    sh_basis(degree, dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2], b);
    const float* c = s_c + t * kw - 3 * k0;
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
        float b[25];
        sh_basis(degree, dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2], b);
        const int nb = (degree + 1) * (degree + 1);
        const float g0 = v_out[3 * i], g1 = v_out[3 * i + 1], g2 = v_out[3 * i + 2];
        float* vc = s_c + t * kw;
        for (int k = 0; k < K; ++k) {
            const float bk = (k + k0 < nb) ? b[k + k0] : 0.0f;
            vc[3 * k] = bk * g0;
            vc[3 * k + 1] = bk * g1;
            vc[3 * k + 2] = bk * g2;
        }
    }
    __syncthreads();
    sh_copy_span(v_coeffs + (size_t)i0 * kw, s_c, cnt * kw);
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
