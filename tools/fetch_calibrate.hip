// fetch_calibrate.hip -- FETCH_SIZE / WRITE_SIZE calibration for the access widths of raster_bwd (VERDICT r02 next #3;
// MI355X_MICROARCH.md HBM section: "other access widths are uncalibrated: calibrate on a known byte count").
//
// Each kernel touches a buffer of KNOWN size exactly once, every 128-B line fully consumed, in one access shape of the
// rasterizer's backward:
//   stream16   global_load_dwordx4, 16 B per lane, coalesced (the guide's reference shape: FETCH_SIZE reads 1/2)
//   sload128   per wave, 128-B records through scalar loads (s_load_dwordx16 x 2): the per-visit record read
//   texel12    buffer_load_dwordx3, 12 B per lane, consecutive lanes on consecutive texels: the texel gathers
//   dword4     global_load_dword, 4 B per lane, coalesced: the sorted-id / slot / cull-word loads
//   store12    global_store_dwordx3, 12 B per lane, 8 lanes per 96-B row: the partial-row stores
//   atomic4    global_atomic_add_f32, 4 B per lane, coalesced, no return: the texel-gradient flush
// Built by tools/gpu_fetchcal.sh into scratch/fetchcal and run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE; each
// kernel prints its byte count, so  factor = bytes / (FETCH_SIZE KiB * 1024)  per shape.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

__global__ void stream16(const float4* __restrict__ src, size_t n4, float* __restrict__ sink) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = src[i];
        acc += (v.x + v.y) + (v.z + v.w);
    }
    if (acc == 12345.678f) sink[0] = acc;  // keeps the loads
}

// one wave per workgroup; wave w reads records w, w + grid, ... with wave-uniform addresses (scalar loads)
__global__ __launch_bounds__(64) void sload128(const float4* __restrict__ rec, size_t n_rec, float* __restrict__ sink) {
    float acc = 0.f;
    for (size_t r = blockIdx.x; r < n_rec; r += gridDim.x) {
        const float4* p = rec + r * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float4 v = p[k];
            acc += (v.x + v.y) + (v.z + v.w);
        }
    }
    if (acc == 12345.678f && threadIdx.x == 0) sink[0] = acc;
}

__global__ void texel12(const float* __restrict__ tex, int n_texels, float* __restrict__ sink) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(tex), 0, n_texels * 12, 0x00020000);
    float acc = 0.f;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n_texels; i += gridDim.x * blockDim.x) {
        const auto t = __builtin_amdgcn_raw_buffer_load_b96(rs, i * 12, 0, 0);
        acc += __int_as_float(t[0]) + __int_as_float(t[1]) + __int_as_float(t[2]);
    }
    if (acc == 12345.678f) sink[0] = acc;
}

__global__ void dword4(const int* __restrict__ src, size_t n, float* __restrict__ sink) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += src[i];
    if (acc == 123456789) sink[0] = (float)acc;
}

struct __attribute__((aligned(4))) F3 { float x, y, z; };
// rows of 24 floats (96 B) at a 128-B stride, written by 8 lanes x 12 B like the backward's partial rows
__global__ void store12(float* __restrict__ rows, size_t n_rows) {
    const int lane = threadIdx.x & 63, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    for (size_t r = wave; r < n_rows; r += nw) {
        if ((lane & 7) == 0) {
            F3* dst = reinterpret_cast<F3*>(rows + r * 32 + 3 * (lane >> 3));
            *dst = F3{1.f, 2.f, (float)lane};
        }
    }
}

__global__ void atomic4(float* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        atomicAdd(dst + i, 1.0f);
}

int main() {
    const size_t bytes = (size_t)1 << 30;  // 1 GiB per buffer: past the 256-MiB Infinity Cache
    char *a, *b;
    float* sink;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(a, 0, bytes));
    CHECK(hipMemset(b, 0, bytes));
    CHECK(hipDeviceSynchronize());
    const int grid = 256 * 32;
    auto flush_caches = [&]() {  // stream the other buffer through L2 / MALL between the measured kernels
        stream16<<<grid, 256>>>((const float4*)b, bytes / 16, sink);
    };
    for (int rep = 0; rep < 3; ++rep) {
        flush_caches();
        stream16<<<grid, 256>>>((const float4*)a, bytes / 16, sink);
        flush_caches();
        sload128<<<256 * 64, 64>>>((const float4*)a, bytes / 128, sink);
        flush_caches();
        const int n_tex = (int)((bytes / 2) / 12);  // 512 MiB of texels (the byte count must fit int32 for the rsrc)
        texel12<<<grid, 256>>>((const float*)a, n_tex, sink);
        flush_caches();
        dword4<<<grid, 256>>>((const int*)a, bytes / 4, sink);
        flush_caches();
        store12<<<grid, 256>>>((float*)a, bytes / 128);
        flush_caches();
        atomic4<<<grid, 256>>>((float*)a, bytes / 8);  // 512 MiB of float atomics
        CHECK(hipDeviceSynchronize());
    }
    std::printf("bytes stream16=%zu sload128=%zu texel12=%zu dword4=%zu store12_rows=%zu(x96B useful, x128B lines) "
                "atomic4=%zu\n", bytes, bytes, (size_t)((bytes / 2) / 12) * 12, bytes, bytes / 128, bytes / 2);
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    CHECK(hipFree(sink));
    return 0;
}
