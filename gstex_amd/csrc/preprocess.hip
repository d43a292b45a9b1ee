// preprocess.hip — per-splat projection, 2DGS screen AABB and tile counts.
//
// Replaces the native ops behind gstex_cuda.get_aabb_2d.{project_points, get_aabb_2d,
// get_num_tiles_hit_2d} (called at nerfstudio/models/gstex.py:1077-1080). One thread per splat;
// every array is SoA-contiguous fp32 so a wave reads 64 consecutive splats per load.
#include "gstex_common.h"
#include "gstex_error.h"
#include "splat_math.h"  // preprocess_splat

using namespace gstex;

namespace {

constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void project_points_kernel(int n, const float* __restrict__ means,
                                                                CamArgs cam_args, float* __restrict__ xys,
                                                                float* __restrict__ depths) {
    const Camera cam = load_camera(cam_args);
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    f3 mu = mk3(means[3 * i], means[3 * i + 1], means[3 * i + 2]);
    float x = vrow(cam, 0, mu) + cam.V[3];
    float y = vrow(cam, 1, mu) + cam.V[7];
    float z = vrow(cam, 2, mu) + cam.V[11];
    depths[i] = z;
    if (z <= kProjClip) {
        xys[2 * i] = 0.0f;
        xys[2 * i + 1] = 0.0f;
        return;
    }
    xys[2 * i] = cam.fx * (x / z) + cam.cx;
    xys[2 * i + 1] = cam.fy * (y / z) + cam.cy;
}

__global__ __launch_bounds__(kBlock) void project_points_bwd_kernel(
    int n, const float* __restrict__ means, CamArgs cam_args, const float* __restrict__ v_xys,
    const float* __restrict__ v_depths, float* __restrict__ v_means) {
    const Camera cam = load_camera(cam_args);
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    f3 mu = mk3(means[3 * i], means[3 * i + 1], means[3 * i + 2]);
    float x = vrow(cam, 0, mu) + cam.V[3];
    float y = vrow(cam, 1, mu) + cam.V[7];
    float z = vrow(cam, 2, mu) + cam.V[11];
    float gx = 0.0f, gy = 0.0f, gz = v_depths ? v_depths[i] : 0.0f;
    if (z > kProjClip && v_xys) {
        float vx = v_xys[2 * i], vy = v_xys[2 * i + 1];
        gx = cam.fx * vx / z;
        gy = cam.fy * vy / z;
        gz = gz - (cam.fx * x * vx + cam.fy * y * vy) / (z * z);
    }
    const float* V = cam.V;
    v_means[3 * i + 0] = (V[0] * gx + V[4] * gy) + V[8] * gz;
    v_means[3 * i + 1] = (V[1] * gx + V[5] * gy) + V[9] * gz;
    v_means[3 * i + 2] = (V[2] * gx + V[6] * gy) + V[10] * gz;
}

__device__ __forceinline__ Homog load_homog(int i, const float* means, const float* scales, float glob,
                                            const float* quats, const Camera& cam, Frame& fr,
                                            float& su, float& sv) {
    fr = quat_frame(quats + 4 * i);
    su = scales[3 * i] * glob;
    sv = scales[3 * i + 1] * glob;
    f3 mu = mk3(means[3 * i], means[3 * i + 1], means[3 * i + 2]);
    return splat_homography(cam, mu, su, sv, fr);
}

__global__ __launch_bounds__(kBlock) void aabb_kernel(int n, const float* __restrict__ means,
                                                      const float* __restrict__ scales, float glob,
                                                      const float* __restrict__ quats, CamArgs cam_args,
                                                      float* __restrict__ centers,
                                                      float* __restrict__ extents) {
    const Camera cam = load_camera(cam_args);
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    Frame fr;
    float su, sv;
    Homog h = load_homog(i, means, scales, glob, quats, cam, fr, su, sv);
    float cx = 0.0f, cy = 0.0f, ex = 0.0f, ey = 0.0f;
    if (!aabb_from_homog(h, cx, cy, ex, ey)) { cx = cy = ex = ey = 0.0f; }
    centers[2 * i] = cx;
    centers[2 * i + 1] = cy;
    extents[2 * i] = ex;
    extents[2 * i + 1] = ey;
}

// d(centre)/d(Tu,Tv,Tw) of aabb_from_homog, then the homography chain to the splat parameters.
__global__ __launch_bounds__(kBlock) void aabb_bwd_kernel(int n, const float* __restrict__ means,
                                                          const float* __restrict__ scales, float glob,
                                                          const float* __restrict__ quats, CamArgs cam_args,
                                                          const float* __restrict__ v_centers,
                                                          float* __restrict__ v_means,
                                                          float* __restrict__ v_scales,
                                                          float* __restrict__ v_quats) {
    const Camera cam = load_camera(cam_args);
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    float gcx = v_centers[2 * i], gcy = v_centers[2 * i + 1];
    Frame fr;
    float su, sv;
    float cx, cy, ex, ey;
    Homog h;
    bool live = !(gcx == 0.0f && gcy == 0.0f);
    if (live) {
        h = load_homog(i, means, scales, glob, quats, cam, fr, su, sv);
        live = aabb_from_homog(h, cx, cy, ex, ey);
    }
    if (!live) {
        // no centre gradient (or a culled splat): the outputs are written, not accumulated
        v_means[3 * i + 0] = v_means[3 * i + 1] = v_means[3 * i + 2] = 0.0f;
        v_scales[3 * i + 0] = v_scales[3 * i + 1] = v_scales[3 * i + 2] = 0.0f;
        v_quats[4 * i + 0] = v_quats[4 * i + 1] = v_quats[4 * i + 2] = v_quats[4 * i + 3] = 0.0f;
        return;
    }
    f3 dTu, dTv, dTw;
    aabb_centre_vjp(h, cx, cy, gcx, gcy, dTu, dTv, dTw);
    HomogGrad g = splat_homography_vjp(cam, su, sv, fr, dTu, dTv, dTw);
    float dq[4];
    frame_vjp(fr, g.dtu, g.dtv, f3{0.0f, 0.0f, 0.0f}, dq);
    v_means[3 * i + 0] = g.dmu.x;
    v_means[3 * i + 1] = g.dmu.y;
    v_means[3 * i + 2] = g.dmu.z;
    v_scales[3 * i + 0] = g.dsu * glob;
    v_scales[3 * i + 1] = g.dsv * glob;
    v_scales[3 * i + 2] = 0.0f;
    v_quats[4 * i + 0] = dq[0];
    v_quats[4 * i + 1] = dq[1];
    v_quats[4 * i + 2] = dq[2];
    v_quats[4 * i + 3] = dq[3];
}

__global__ __launch_bounds__(kBlock) void num_tiles_kernel(int n, const float* __restrict__ centers,
                                                           const float* __restrict__ extents, int tiles_x,
                                                           int tiles_y, int block,
                                                           int32_t* __restrict__ out) {
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    Rect r = tile_rect(centers[2 * i], centers[2 * i + 1], extents[2 * i], extents[2 * i + 1], tiles_x,
                       tiles_y, block);
    out[i] = (r.x1 - r.x0) * (r.y1 - r.y0);
}

// The three preprocessing outputs the raster needs, in one pass over the splats (the training path calls them
// back to back on the same inputs): view depth as project_points_kernel, centre / extent as aabb_kernel and the
// tile count as num_tiles_kernel compute them -- the same device functions, so bit-identical.
__global__ __launch_bounds__(kBlock) void preprocess_kernel(int n, const float* __restrict__ means,
                                                            const float* __restrict__ scales, float glob,
                                                            const float* __restrict__ quats, CamArgs cam_args,
                                                            int tiles_x, int tiles_y, int block,
                                                            float* __restrict__ depths, float* __restrict__ centers,
                                                            float* __restrict__ extents, int32_t* __restrict__ nth) {
    const Camera cam = load_camera(cam_args);
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const Preprocessed p = preprocess_splat(cam, mk3(means[3 * i], means[3 * i + 1], means[3 * i + 2]), scales[3 * i],
                                            scales[3 * i + 1], glob, quats + 4 * i, tiles_x, tiles_y, block);
    depths[i] = p.depth;
    centers[2 * i] = p.cx;
    centers[2 * i + 1] = p.cy;
    extents[2 * i] = p.ex;
    extents[2 * i + 1] = p.ey;
    nth[i] = p.nth;
}

}  // namespace

extern "C" int gstex_preprocess(int32_t n, const float* means, const float* scales, float glob_scale,
                                const float* quats, const gstex_camera* cam, float* depths, float* centers,
                                float* extents, int32_t* num_tiles_hit, void* stream) {
    GSTEX_REQUIRE(n >= 0 && cam && cam->H >= 0 && cam->W >= 0 && cam->block > 0, "gstex_preprocess: invalid arguments");
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(means && scales && quats && depths && centers && extents && num_tiles_hit,
                  "gstex_preprocess: null pointer");
    const int tx = (cam->W + cam->block - 1) / cam->block, ty = (cam->H + cam->block - 1) / cam->block;
    preprocess_kernel<<<div_up(n, kBlock), kBlock, 0, as_stream(stream)>>>(
        n, means, scales, glob_scale, quats, to_device_camera(*cam), tx, ty, cam->block, depths, centers, extents,
        num_tiles_hit);
    return launch_status("gstex_preprocess");
}

extern "C" int gstex_project_points(int32_t n, const float* means, const gstex_camera* cam, float* xys,
                                    float* depths, void* stream) {
    GSTEX_REQUIRE(n >= 0 && cam, "gstex_project_points: invalid arguments");
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(means && xys && depths, "gstex_project_points: null pointer");
    project_points_kernel<<<div_up(n, kBlock), kBlock, 0, as_stream(stream)>>>(
        n, means, to_device_camera(*cam), xys, depths);
    return launch_status("gstex_project_points");
}

extern "C" int gstex_project_points_bwd(int32_t n, const float* means, const gstex_camera* cam,
                                        const float* v_xys, const float* v_depths, float* v_means,
                                        void* stream) {
    GSTEX_REQUIRE(n >= 0 && cam, "gstex_project_points_bwd: invalid arguments");
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(means && v_means, "gstex_project_points_bwd: null pointer");
    project_points_bwd_kernel<<<div_up(n, kBlock), kBlock, 0, as_stream(stream)>>>(
        n, means, to_device_camera(*cam), v_xys, v_depths, v_means);
    return launch_status("gstex_project_points_bwd");
}

extern "C" int gstex_aabb_2d(int32_t n, const float* means, const float* scales, float glob_scale,
                             const float* quats, const gstex_camera* cam, float* centers, float* extents,
                             void* stream) {
    GSTEX_REQUIRE(n >= 0 && cam, "gstex_aabb_2d: invalid arguments");
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(means && scales && quats && centers && extents, "gstex_aabb_2d: null pointer");
    aabb_kernel<<<div_up(n, kBlock), kBlock, 0, as_stream(stream)>>>(n, means, scales, glob_scale, quats,
                                                                      to_device_camera(*cam), centers,
                                                                      extents);
    return launch_status("gstex_aabb_2d");
}

extern "C" int gstex_aabb_2d_bwd(int32_t n, const float* means, const float* scales, float glob_scale,
                                 const float* quats, const gstex_camera* cam, const float* v_centers,
                                 float* v_means, float* v_scales, float* v_quats, void* stream) {
    GSTEX_REQUIRE(n >= 0 && cam, "gstex_aabb_2d_bwd: invalid arguments");
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(means && scales && quats && v_centers && v_means && v_scales && v_quats,
                  "gstex_aabb_2d_bwd: null pointer");
    aabb_bwd_kernel<<<div_up(n, kBlock), kBlock, 0, as_stream(stream)>>>(
        n, means, scales, glob_scale, quats, to_device_camera(*cam), v_centers, v_means, v_scales, v_quats);
    return launch_status("gstex_aabb_2d_bwd");
}

extern "C" int gstex_num_tiles_hit(int32_t n, const float* centers, const float* extents, int32_t H,
                                   int32_t W, int32_t block, int32_t* num_tiles_hit, void* stream) {
    GSTEX_REQUIRE(n >= 0 && H >= 0 && W >= 0 && block > 0, "gstex_num_tiles_hit: invalid arguments");
    if (n == 0) return GSTEX_OK;
    GSTEX_REQUIRE(centers && extents && num_tiles_hit, "gstex_num_tiles_hit: null pointer");
    int tx = (W + block - 1) / block, ty = (H + block - 1) / block;
    num_tiles_kernel<<<div_up(n, kBlock), kBlock, 0, as_stream(stream)>>>(n, centers, extents, tx, ty, block,
                                                                           num_tiles_hit);
    return launch_status("gstex_num_tiles_hit");
}
