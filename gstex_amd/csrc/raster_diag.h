// raster_diag.h — diagnostic counters of the raster kernels, compiled in only by diagnostic builds
// (tools/build_variant.sh EXTRA=-DGSTEX_STATS=1 / =3, read back by tools/gpu_stats.sh and tools/wg_timeline.py).
// The product build (GSTEX_STATS = 0) defines every hook below as an empty statement.
//   GSTEX_STAT(i, v)   add v to counter i from the wave's lane 0 (wave-uniform code)
//   GSTEX_STATW(i, v)  the same from the first active lane (divergent code)
//   GSTEX_WG_STAMP(depth, wl)  GSTEX_STATS == 3: per-workgroup timeline (start / end s_memrealtime, tile depth, last
//                              contributor) for the first 65536 workgroups
#pragma once
#ifndef GSTEX_STATS
#define GSTEX_STATS 0
#endif
#if GSTEX_STATS
__device__ unsigned long long g_stats[24];  // [0, 8) backward, [8, 13) forward counters, [13, 16) backward
extern "C" int gstex_debug_stats(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stats), sizeof(g_stats)) == hipSuccess ? 0 : 2;
}
__device__ unsigned long long g_wg[65536 * 4];
extern "C" int gstex_debug_wg(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wg), sizeof(g_wg)) == hipSuccess ? 0 : 2;
}
#endif
#if GSTEX_STATS == 1
#define GSTEX_STAT(i, v) do { const unsigned long long v_ = (v); if ((threadIdx.x & 63) == 0) atomicAdd(&g_stats[i], v_); } while (0)
#define GSTEX_STATW(i, v) do { const unsigned long long v_ = (v); \
    if ((int)(threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) atomicAdd(&g_stats[i], v_); } while (0)
#else
#define GSTEX_STAT(i, v) do { } while (0)
#define GSTEX_STATW(i, v) do { } while (0)
#endif
#if GSTEX_STATS == 3
struct GstexWgStamp {
    unsigned long long t0;
    int depth, wl;
    __device__ ~GstexWgStamp() {
        if (threadIdx.x == 0 && blockIdx.x < 65536) {
            g_wg[4 * blockIdx.x] = t0;
            g_wg[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
            g_wg[4 * blockIdx.x + 2] = (unsigned long long)depth;
            g_wg[4 * blockIdx.x + 3] = (unsigned long long)(long long)wl;
        }
    }
};
#define GSTEX_WG_STAMP(depth, wl) GstexWgStamp stamp_{__builtin_amdgcn_s_memrealtime(), (depth), (wl)}
#else
#define GSTEX_WG_STAMP(depth, wl) do { } while (0)
#endif
// GSTEX_PAIR_DUMP (tools/hp_pairs.py): every contributing pair of the backward appends one 16-float record
//   gid (bits), px, py, flags (use3 | aclamp << 1, bits), T, w, dL/dalpha, drho, u, v, 1 / p.z, z, alpha, G, dx, dy
// to the buffer gstex_debug_pair_dump installed (vector atomics on the count; records past `cap` are dropped).
#ifdef GSTEX_PAIR_DUMP
__device__ float* g_pair_buf;
__device__ int* g_pair_count;
__device__ int g_pair_cap;
extern "C" int gstex_debug_pair_dump(float* buf, int cap, int* count) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_pair_buf), &buf, sizeof(buf)) != hipSuccess) return 2;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_pair_count), &count, sizeof(count)) != hipSuccess) return 2;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_pair_cap), &cap, sizeof(cap)) == hipSuccess ? 0 : 2;
}
#define GSTEX_PAIR(...) do { \
    const float v_[16] = {__VA_ARGS__}; \
    if (g_pair_buf) { const int k_ = atomicAdd(g_pair_count, 1); \
        if (k_ < g_pair_cap) for (int i_ = 0; i_ < 16; ++i_) g_pair_buf[16 * (size_t)k_ + i_] = v_[i_]; } } while (0)
#else
#define GSTEX_PAIR(...) do { } while (0)
#endif
