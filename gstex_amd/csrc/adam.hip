// adam.hip — one-launch multi-tensor Adam for the GStex parameter groups.
//
//   gstex_adam_step   <- torch.optim.Adam(eps=1e-15) over the 7 GStex parameter groups
//                        (gstex_configs.py:207-244 via engine/optimizers.py:158-171).
//
// Per element, in torch's foreach-Adam order (torch/optim/adam.py _multi_tensor_adam):
//   m = lerp(m, g, 1 - beta1)                      m + (1-beta1) * (g - m)
//   v = v * beta2 + (1 - beta2) * (g * g)
//   p = p - step_size * m / (sqrt(v) / sqrt(bc2) + eps),  step_size = lr / bc1
// with bc1 = 1 - beta1^t, bc2 = 1 - beta2^t computed on the host per tensor (each tensor keeps its own step
// count; a rechart zeroes the texel store's moments m and v and keeps its step count, like the reference's
// reshape_in_optim, gstex.py:809-815 -- GStexTrainer.recharge).
// HBM-bound: 16 B read + 12 B written per element, float4 vectorised, one launch for all tensors; one
// float4 per thread with nontemporal loads/stores (measured at cfg3: 205 us with 4 cached float4 per
// thread, 178 us like this = 6.5 TB/s).
#include "gstex_common.h"
#include "gstex_error.h"

namespace {

constexpr int kAdamThreads = 256;
#ifndef GSTEX_ADAM_VEC
#define GSTEX_ADAM_VEC 1
#endif
#ifndef GSTEX_ADAM_NT
#define GSTEX_ADAM_NT 1
#endif
constexpr int kAdamVec = GSTEX_ADAM_VEC;  // float4 per thread
constexpr int kAdamPerBlock = kAdamThreads * 4 * kAdamVec;
constexpr int kAdamMaxTensors = GSTEX_ADAM_MAX_TENSORS;

// streaming accesses: every byte is touched once per step, so nothing is worth keeping in the caches
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_stream(const float4* p) {
    if (!GSTEX_ADAM_NT) return *p;
    const f4v x = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return make_float4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ void st_stream(float4* p, const float4& x) {
    if (!GSTEX_ADAM_NT) { *p = x; return; }
    const f4v y = {x.x, x.y, x.z, x.w};
    __builtin_nontemporal_store(y, reinterpret_cast<f4v*>(p));
}

struct AdamArgs {
    gstex_adam_tensor t[kAdamMaxTensors];
    int64_t block_start[kAdamMaxTensors + 1];
    int n;
    float beta1, beta2, eps, one_m_beta1, one_m_beta2;
    float gscale;  // gradient scale applied on read (gstex_adam_step_scaled: a data-parallel 1 / world), 1 = none
    const float* skip;  // gstex_adam_step_guarded: nothing is updated when *skip != 0 (nullable)
};

template <bool SCALE>
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float b1w, float b2,
                                          float one_m_b2, float eps, float neg_step, float bc2_sqrt, float gs) {
    if (SCALE) g = g * gs;  // the same fp32 product as scaling the gradient buffer first
    m = m + b1w * (g - m);
    v = v * b2 + one_m_b2 * (g * g);
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = p + neg_step * (m / denom);
}

// ZERO_GRAD: the gradient is zeroed after it is read (the next backward accumulates into the same buffer: no separate
// fill launch, and the zeroing rides along with an update that may run on a side stream)
template <bool ZERO_GRAD, bool SCALE>
__device__ __forceinline__ void adam_chunk(const AdamArgs& a, const int64_t b) {
    int k = 0;
    while (k + 1 < a.n && a.block_start[k + 1] <= b) ++k;
    const gstex_adam_tensor& t = a.t[k];
    const int64_t base = (b - a.block_start[k]) * kAdamPerBlock;
    const float neg_step = -t.step_size, bc2s = t.bias_correction2_sqrt;
    const bool vec = ((reinterpret_cast<uintptr_t>(t.param) | reinterpret_cast<uintptr_t>(t.grad) |
                       reinterpret_cast<uintptr_t>(t.exp_avg) | reinterpret_cast<uintptr_t>(t.exp_avg_sq)) & 15) == 0;
    if (vec) {
        // all 4 * kAdamVec loads of the thread issued before any store (stores could alias later loads, so the
        // compiler would otherwise keep only one iteration's 4 loads in flight)
        float4 p[kAdamVec], g[kAdamVec], m[kAdamVec], v[kAdamVec];
        bool full[kAdamVec];
#pragma unroll
        for (int r = 0; r < kAdamVec; ++r) {
            const int64_t i = base + 4 * ((int64_t)r * kAdamThreads + threadIdx.x);
            full[r] = i + 3 < t.numel;
            if (full[r]) {
                p[r] = ld_stream(reinterpret_cast<const float4*>(t.param + i));
                g[r] = ld_stream(reinterpret_cast<const float4*>(t.grad + i));
                m[r] = ld_stream(reinterpret_cast<const float4*>(t.exp_avg + i));
                v[r] = ld_stream(reinterpret_cast<const float4*>(t.exp_avg_sq + i));
            }
        }
#pragma unroll
        for (int r = 0; r < kAdamVec; ++r) {
            const int64_t i = base + 4 * ((int64_t)r * kAdamThreads + threadIdx.x);
            if (full[r]) {
                adam_elem<SCALE>(p[r].x, g[r].x, m[r].x, v[r].x, a.one_m_beta1, a.beta2, a.one_m_beta2, a.eps, neg_step, bc2s, a.gscale);
                adam_elem<SCALE>(p[r].y, g[r].y, m[r].y, v[r].y, a.one_m_beta1, a.beta2, a.one_m_beta2, a.eps, neg_step, bc2s, a.gscale);
                adam_elem<SCALE>(p[r].z, g[r].z, m[r].z, v[r].z, a.one_m_beta1, a.beta2, a.one_m_beta2, a.eps, neg_step, bc2s, a.gscale);
                adam_elem<SCALE>(p[r].w, g[r].w, m[r].w, v[r].w, a.one_m_beta1, a.beta2, a.one_m_beta2, a.eps, neg_step, bc2s, a.gscale);
                st_stream(reinterpret_cast<float4*>(t.param + i), p[r]);
                st_stream(reinterpret_cast<float4*>(t.exp_avg + i), m[r]);
                st_stream(reinterpret_cast<float4*>(t.exp_avg_sq + i), v[r]);
                if (ZERO_GRAD) st_stream(reinterpret_cast<float4*>(const_cast<float*>(t.grad) + i), make_float4(0.f, 0.f, 0.f, 0.f));
            } else {
                for (int64_t e = i; e < t.numel; ++e) {
                    adam_elem<SCALE>(t.param[e], t.grad[e], t.exp_avg[e], t.exp_avg_sq[e], a.one_m_beta1, a.beta2,
                                     a.one_m_beta2, a.eps, neg_step, bc2s, a.gscale);
                    if (ZERO_GRAD) const_cast<float*>(t.grad)[e] = 0.0f;
                }
            }
        }
    } else {
        for (int e = threadIdx.x; e < kAdamPerBlock; e += kAdamThreads) {
            const int64_t i = base + e;
            if (i < t.numel) {
                adam_elem<SCALE>(t.param[i], t.grad[i], t.exp_avg[i], t.exp_avg_sq[i], a.one_m_beta1, a.beta2,
                                 a.one_m_beta2, a.eps, neg_step, bc2s, a.gscale);
                if (ZERO_GRAD) const_cast<float*>(t.grad)[i] = 0.0f;
            }
        }
    }
}

// grid-stride over the chunks: a capped grid (GSTEX_ADAM_GRID flags) leaves most of every CU to another stream
template <bool ZERO_GRAD, bool SCALE>
__global__ __launch_bounds__(kAdamThreads) void adam_kernel(const AdamArgs a) {
    if (a.skip && *a.skip != 0.0f) return;  // an overflowed step (pair-capacity guard): no update
    for (int64_t b = blockIdx.x; b < a.block_start[a.n]; b += gridDim.x) adam_chunk<ZERO_GRAD, SCALE>(a, b);
}

}  // namespace

namespace {
int adam_launch(int32_t n_tensors, const gstex_adam_tensor* tensors, double beta1, double beta2, double eps,
                int32_t flags, float grad_scale, void* stream, const float* skip = nullptr) {
    GSTEX_REQUIRE(n_tensors >= 0 && n_tensors <= kAdamMaxTensors,
                  "gstex_adam_step: n_tensors must be in [0, %d] (got %d)", kAdamMaxTensors, n_tensors);
    GSTEX_REQUIRE(n_tensors == 0 || tensors, "gstex_adam_step: null tensor table");
    AdamArgs a{};
    int64_t blocks = 0;
    int k = 0;
    for (int i = 0; i < n_tensors; ++i) {
        const gstex_adam_tensor& t = tensors[i];
        GSTEX_REQUIRE(t.numel >= 0, "gstex_adam_step: tensor %d has numel < 0", i);
        if (t.numel == 0) continue;
        GSTEX_REQUIRE(t.param && t.grad && t.exp_avg && t.exp_avg_sq, "gstex_adam_step: tensor %d: null pointer", i);
        a.t[k] = t;
        a.block_start[k] = blocks;
        blocks += (t.numel + kAdamPerBlock - 1) / kAdamPerBlock;
        ++k;
    }
    if (k == 0) return GSTEX_OK;
    a.block_start[k] = blocks;
    a.n = k;
    // scalars rounded to fp32 from double, as torch passes its python-float hyper-parameters
    a.beta1 = (float)beta1;
    a.beta2 = (float)beta2;
    a.eps = (float)eps;
    a.one_m_beta1 = (float)(1.0 - beta1);
    a.one_m_beta2 = (float)(1.0 - beta2);
    a.gscale = grad_scale;
    a.skip = skip;
    const int64_t cap = (flags >> GSTEX_ADAM_GRID_SHIFT) & 0xFFFF;
    const unsigned grid = (unsigned)(cap > 0 && cap < blocks ? cap : blocks);
    const hipStream_t st = gstex::as_stream(stream);
    const bool zg = flags & GSTEX_ADAM_ZERO_GRAD, sc = grad_scale != 1.0f;
    if (zg && sc) adam_kernel<true, true><<<grid, kAdamThreads, 0, st>>>(a);
    else if (zg) adam_kernel<true, false><<<grid, kAdamThreads, 0, st>>>(a);
    else if (sc) adam_kernel<false, true><<<grid, kAdamThreads, 0, st>>>(a);
    else adam_kernel<false, false><<<grid, kAdamThreads, 0, st>>>(a);
    return gstex::launch_status("gstex_adam_step");
}
}  // namespace

extern "C" int gstex_adam_step(int32_t n_tensors, const gstex_adam_tensor* tensors, double beta1, double beta2,
                               double eps, void* stream) {
    return adam_launch(n_tensors, tensors, beta1, beta2, eps, 0, 1.0f, stream);
}

extern "C" int gstex_adam_step_ex(int32_t n_tensors, const gstex_adam_tensor* tensors, double beta1, double beta2,
                                  double eps, int32_t flags, void* stream) {
    GSTEX_REQUIRE((flags & ~(GSTEX_ADAM_ZERO_GRAD | (0xFFFF << GSTEX_ADAM_GRID_SHIFT))) == 0,
                  "gstex_adam_step_ex: unknown flags 0x%x", flags);
    return adam_launch(n_tensors, tensors, beta1, beta2, eps, flags, 1.0f, stream);
}

extern "C" int gstex_adam_step_scaled(int32_t n_tensors, const gstex_adam_tensor* tensors, double beta1, double beta2,
                                      double eps, int32_t flags, float grad_scale, void* stream) {
    GSTEX_REQUIRE((flags & ~(GSTEX_ADAM_ZERO_GRAD | (0xFFFF << GSTEX_ADAM_GRID_SHIFT))) == 0,
                  "gstex_adam_step_scaled: unknown flags 0x%x", flags);
    GSTEX_REQUIRE(grad_scale == grad_scale && grad_scale > 0.0f && grad_scale <= 1.0f,
                  "gstex_adam_step_scaled: grad_scale must be in (0, 1] (got %g)", (double)grad_scale);
    return adam_launch(n_tensors, tensors, beta1, beta2, eps, flags, grad_scale, stream);
}

extern "C" int gstex_adam_step_guarded(int32_t n_tensors, const gstex_adam_tensor* tensors, double beta1, double beta2,
                                       double eps, int32_t flags, float grad_scale, const float* skip, void* stream) {
    GSTEX_REQUIRE((flags & ~(GSTEX_ADAM_ZERO_GRAD | (0xFFFF << GSTEX_ADAM_GRID_SHIFT))) == 0,
                  "gstex_adam_step_guarded: unknown flags 0x%x", flags);
    GSTEX_REQUIRE(grad_scale == grad_scale && grad_scale > 0.0f && grad_scale <= 1.0f,
                  "gstex_adam_step_guarded: grad_scale must be in (0, 1] (got %g)", (double)grad_scale);
    return adam_launch(n_tensors, tensors, beta1, beta2, eps, flags, grad_scale, stream, skip);
}
