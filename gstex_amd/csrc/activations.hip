// activations.hip — per-step splat parameter activations and UV frames, fused.
//
//   gstex_activate_fwd / gstex_activate_bwd  <- GStexModel.get_outputs (gstex.py:1059-1066, 975-990,
//                                               1101-1104), one thread per splat:
//     quats     = q / |q|
//     scales    = [clamp(exp(s0), 1e-9), clamp(exp(s1), 1e-9), 1e-5 * mean(those two) (detached)]
//     opacities = sigmoid(o)
//     uv0 = 0.5, umap = m0 * R(q')[:, 0], vmap = m1 * R(q')[:, 1]   (q' = normalize(quats), detached)
//     viewdirs  = (means - campos) / |means - campos|               (detached)
//   The backward carries the three differentiable paths: the quaternion normalisation
//   (v_q = (v_qn - qn (qn . v_qn)) / |q|), exp with the clamp mask for the first two scale axes
//   (the third is detached), and the sigmoid.  Replaces ~40 small torch kernels per step.
#include "gstex_common.h"
#include "gstex_error.h"
#include "splat_math.h"  // activate_splat

using namespace gstex;

namespace {

__device__ __forceinline__ float norm4(float a, float b, float c, float d) {
    return sqrtf(((a * a + b * b) + c * c) + d * d);
}

__global__ __launch_bounds__(256) void activate_fwd_kernel(
    int n, const float* __restrict__ means, const float* __restrict__ quats, const float* __restrict__ log_scales,
    const float* __restrict__ opac_logits, const float* __restrict__ mappings, int map_stride,
    const float* __restrict__ campos, float* __restrict__ quats_n, float* __restrict__ scales,
    float* __restrict__ opacities, float* __restrict__ uv0, float* __restrict__ umap, float* __restrict__ vmap,
    float* __restrict__ viewdirs) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const Activated a = activate_splat(reinterpret_cast<const float4*>(quats)[i], log_scales[3 * i],
                                       log_scales[3 * i + 1], opac_logits[i], mappings[(size_t)map_stride * i],
                                       mappings[(size_t)map_stride * i + 1], means[3 * i], means[3 * i + 1],
                                       means[3 * i + 2], campos);
    store_activated(i, a, quats_n, scales, opacities, uv0, umap, vmap, viewdirs);
}

__global__ __launch_bounds__(256) void activate_bwd_kernel(
    int n, const float* __restrict__ quats, const float* __restrict__ log_scales,
    const float* __restrict__ opacities, const float* __restrict__ v_quats_n, const float* __restrict__ v_scales,
    const float* __restrict__ v_opacities, float* __restrict__ v_quats, float* __restrict__ v_log_scales,
    float* __restrict__ v_opac_logits) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 g = v_quats_n ? reinterpret_cast<const float4*>(v_quats_n)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float gs0 = v_scales ? v_scales[3 * i] : 0.f, gs1 = v_scales ? v_scales[3 * i + 1] : 0.f;
    const float go = v_opacities ? v_opacities[i] : 0.f;
    float4 vq;
    float vls0, vls1, vo;
    // (the function evaluates all three; a null output skips its loads' use only)
    activate_bwd_splat(reinterpret_cast<const float4*>(quats)[i], log_scales[3 * i], log_scales[3 * i + 1],
                       opacities[i], g, gs0, gs1, go, vq, vls0, vls1, vo);
    if (v_quats) reinterpret_cast<float4*>(v_quats)[i] = vq;
    if (v_log_scales) {
        v_log_scales[3 * i] = vls0;
        v_log_scales[3 * i + 1] = vls1;
        v_log_scales[3 * i + 2] = 0.0f;  // the third axis is 1e-5 * mean(...).detach()
    }
    if (v_opac_logits) v_opac_logits[i] = vo;
}

}  // namespace

extern "C" int gstex_activate_fwd(int32_t n, const float* means, const float* quats, const float* log_scales,
                                  const float* opac_logits, const float* mappings, int32_t mappings_stride,
                                  const float* campos, float* quats_n, float* scales, float* opacities, float* uv0,
                                  float* umap, float* vmap, float* viewdirs, void* stream) {
    GSTEX_REQUIRE(n >= 0 && mappings_stride >= 2, "gstex_activate_fwd: invalid sizes (n=%d, mappings_stride=%d)", n,
                  mappings_stride);
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(means && quats && log_scales && opac_logits && mappings && campos && quats_n && scales && opacities &&
                      uv0 && umap && vmap && viewdirs,
                  "gstex_activate_fwd: null pointer");
    GSTEX_REQUIRE(((reinterpret_cast<uintptr_t>(quats) | reinterpret_cast<uintptr_t>(quats_n)) & 15) == 0,
                  "gstex_activate_fwd: quaternions must be 16-byte aligned");
    activate_fwd_kernel<<<div_up(n, 256), 256, 0, as_stream(stream)>>>(n, means, quats, log_scales, opac_logits,
                                                                        mappings, mappings_stride, campos, quats_n,
                                                                        scales, opacities, uv0, umap, vmap, viewdirs);
    return launch_status("gstex_activate_fwd");
}

extern "C" int gstex_activate_bwd(int32_t n, const float* quats, const float* log_scales, const float* opacities,
                                  const float* v_quats_n, const float* v_scales, const float* v_opacities,
                                  float* v_quats, float* v_log_scales, float* v_opac_logits, void* stream) {
    GSTEX_REQUIRE(n >= 0, "gstex_activate_bwd: n < 0");
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(quats && log_scales && opacities, "gstex_activate_bwd: null pointer");
    GSTEX_REQUIRE(((reinterpret_cast<uintptr_t>(quats) | reinterpret_cast<uintptr_t>(v_quats) |
                    reinterpret_cast<uintptr_t>(v_quats_n)) & 15) == 0,
                  "gstex_activate_bwd: quaternions must be 16-byte aligned");
    activate_bwd_kernel<<<div_up(n, 256), 256, 0, as_stream(stream)>>>(n, quats, log_scales, opacities, v_quats_n,
                                                                        v_scales, v_opacities, v_quats, v_log_scales,
                                                                        v_opac_logits);
    return launch_status("gstex_activate_bwd");
}
