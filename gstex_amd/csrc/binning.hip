// binning.hip — tile binning and per-tile depth sort (the sort that happens inside the reference's
// texture_gaussians, args at nerfstudio/models/gstex.py:1136-1139,1158).
//
// Output order is the gsplat-0.1 lineage order: per tile, splats ascending by (depth float bits,
// splat id) — what a stable radix sort of (tile << 32 | depth_bits) over gid-major emitted pairs
// produces.  The MI355X design does not run a 64-bit global radix sort; instead:
//   1. count:  per splat, one returning atomic per covered tile gives the pair its rank in the
//              tile bucket (order inside a bucket is arbitrary at this point);
//   2. scan:   exclusive scan of the per-tile counts -> tile ranges;
//   3. place:  each pair writes its 64-bit key (depth_bits << 32 | id) to start[tile] + rank;
//   4. sort:   one workgroup per tile sorts its bucket in LDS (bitonic, power-of-two padded);
//              buckets larger than the LDS capacity are chunk-sorted in LDS and merged in global
//              memory with merge-path by the same workgroup.
// Keys are unique (id is part of the key), so any correct sort yields the same, bit-exact order.
#include "gstex_common.h"
#include "gstex_error.h"
#include "gstex_internal.h"
#include "splat_math.h"

using namespace gstex;

namespace {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 4;
constexpr int kScanTile = kScanThreads * kScanItems;
constexpr int kSortThreads = 256;
constexpr int kSortCap = 4096;  // keys per LDS sort (32 KiB)
#ifndef GSTEX_SORT_REGS
#define GSTEX_SORT_REGS 1
#endif

__global__ __launch_bounds__(kScanThreads) void scan_partials_kernel(int n, const int32_t* __restrict__ in,
                                                                     int32_t* __restrict__ block_sums) {
    __shared__ int s_wave[kScanThreads / 64];
    int base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    int v = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) v += (base + k < n) ? in[base + k] : 0;
    int total;
    block_excl_scan<kScanThreads>(v, s_wave, &total);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = total;
}

// Single block: exclusive scan of the block sums in place.
__global__ __launch_bounds__(kScanThreads) void scan_block_sums_kernel(int nb, int32_t* __restrict__ sums) {
    __shared__ int s_wave[kScanThreads / 64];
    int carry = 0;
    for (int b0 = 0; b0 < nb; b0 += kScanThreads) {
        int i = b0 + threadIdx.x;
        int v = (i < nb) ? sums[i] : 0;
        int total;
        int ex = block_excl_scan<kScanThreads>(v, s_wave, &total);
        if (i < nb) sums[i] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(kScanThreads) void scan_final_kernel(int n, const int32_t* __restrict__ in,
                                                                  const int32_t* __restrict__ block_offs,
                                                                  int32_t* __restrict__ out, const ScanGuard guard) {
    __shared__ int s_wave[kScanThreads / 64];
    int base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    int vals[kScanItems];
    int v = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        vals[k] = (base + k < n) ? in[base + k] : 0;
        v += vals[k];
    }
    int total;
    int ex = block_excl_scan<kScanThreads>(v, s_wave, &total) + block_offs[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        if (base + k < n) out[base + k] = ex;
        ex += vals[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kScanThreads - 1) {
        out[n] = ex;
        apply_guard(guard, ex);
    }
}

// Short inputs (the per-tile scans): one workgroup walks the tiles with a running carry, one launch instead of three.
__global__ __launch_bounds__(kScanThreads) void scan_single_kernel(int n, const int32_t* __restrict__ in,
                                                                   int32_t* __restrict__ out, const ScanGuard guard) {
    __shared__ int s_wave[kScanThreads / 64];
    int carry = 0;
    for (int b0 = 0; b0 < n; b0 += kScanTile) {
        const int base = b0 + threadIdx.x * kScanItems;
        int vals[kScanItems];
        int v = 0;
#pragma unroll
        for (int k = 0; k < kScanItems; ++k) {
            vals[k] = (base + k < n) ? in[base + k] : 0;
            v += vals[k];
        }
        int total;
        int ex = block_excl_scan<kScanThreads>(v, s_wave, &total) + carry;
#pragma unroll
        for (int k = 0; k < kScanItems; ++k) {
            if (base + k < n) out[base + k] = ex;
            ex += vals[k];
        }
        carry += total;
    }
    if (threadIdx.x == 0) {
        out[n] = carry;
        apply_guard(guard, carry);
    }
}
constexpr int kScanSingleMaxTiles = 16;

int run_scan(int n, const int32_t* in, int32_t* out, int32_t* block_sums, hipStream_t st,
             const ScanGuard guard = ScanGuard{0, nullptr, nullptr, 0}) {
    int nb = div_up(n, kScanTile);
    if (nb <= kScanSingleMaxTiles) {  // (n = 0 included: the single workgroup writes out[0] = 0)
        scan_single_kernel<<<1, kScanThreads, 0, st>>>(n, in, out, guard);
        return launch_status("scan");
    }
    scan_partials_kernel<<<nb, kScanThreads, 0, st>>>(n, in, block_sums);
    scan_block_sums_kernel<<<1, kScanThreads, 0, st>>>(nb, block_sums);
    scan_final_kernel<<<nb, kScanThreads, 0, st>>>(n, in, block_sums, out, guard);
    return launch_status("scan");
}

size_t scan_ws_bytes(int n) { return (size_t)(div_up(n, kScanTile) + 1) * sizeof(int32_t); }

// 1. count + rank
// Capacity mode (gstex_bin_sort_capped): the pair total offsets[n] is read on the device; a total beyond the pair
// buffers' capacity leaves every tile empty (no pair is emitted, so nothing is written past the buffers) and the
// step's guard flag (gstex_scan_offsets_guarded) tells the optimizer to skip the step.
__device__ __forceinline__ bool over_capacity(const int32_t* offsets, int n, long long cap) {
    return cap >= 0 && (long long)offsets[n] > cap;
}

__global__ __launch_bounds__(256) void count_kernel(int n, const float* __restrict__ centers,
                                                    const float* __restrict__ extents,
                                                    const int32_t* __restrict__ offsets, int tiles_x,
                                                    int tiles_y, int block, int32_t* __restrict__ tile_count,
                                                    int32_t* __restrict__ rank, long long cap) {
    if (over_capacity(offsets, n, cap)) return;
    int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= n) return;
    Rect r = tile_rect(centers[2 * g], centers[2 * g + 1], extents[2 * g], extents[2 * g + 1], tiles_x,
                       tiles_y, block);
    int e = offsets[g];
    for (int ty = r.y0; ty < r.y1; ++ty)
        for (int tx = r.x0; tx < r.x1; ++tx) rank[e++] = atomicAdd(&tile_count[ty * tiles_x + tx], 1);
}

// 1'. the same count + rank with the tile histogram privatised in LDS: each workgroup builds the histogram of its
// 256 * kCountSplatsPerThread splats' pairs with LDS atomics, reserves one global range per touched tile (one global
// atomic per (workgroup, tile) instead of one per pair: the image centre's tiles receive ~2000 pairs each, which
// serialised on their counters), then ranks each pair inside its tile's range with a second LDS atomic.  (The
// earlier form ranked first and added the range start with a global read-modify-write per pair afterwards: a serial
// chain of global loads per thread, 45 -> 28 us at cfg3 without it.)  Ranks are scattered positions inside a tile's
// bucket only; the per-tile sort by (depth, id) makes the final order independent of them.
#ifndef GSTEX_COUNT_SPT
#define GSTEX_COUNT_SPT 2  // splats per thread (measured at cfg3: 4 -> 2 saves 5 us, 1 is slower: more range reservations)
#endif
constexpr int kCountSplatsPerThread = GSTEX_COUNT_SPT;
#ifndef GSTEX_COUNT_RESERVE
#define GSTEX_COUNT_RESERVE 1  // histogram, reserve, then rank (no global read-modify-write of the ranks)
#endif
constexpr int kCountLdsTiles = 16384;  // 64 KiB histogram

#ifndef GSTEX_WAVE_PAIRS
#define GSTEX_WAVE_PAIRS 1
#endif
// place_kernel: wave-cooperative walk over the (splat, tile) pairs of 64 consecutive splats (lane l <-> splat l): the
// pairs occupy the contiguous emission range [e0 of lane 0, e0 + count of lane 63) and lane l of the
// wave takes pairs l, l + 64, ... of it, so a large splat's tiles are spread over the whole wave (no
// lane runs its splat's loop alone while the others idle) and the rank / slot writes are coalesced.
// The owner of pair e is the last lane whose first slot is <= e (lanes without a splat carry INT_MAX).
// Must be called with every lane of the wave active (the shuffles read all lanes).  Not used by the
// count: there one LDS atomic per pair is cheaper than the owner search's ten lane shuffles (measured
// 46 -> 60 us at cfg3), while the place kernel's scattered global stores hide them (47 -> 32 us).
struct WavePairs {
    int e0, x0, y0, w, g;
};
__device__ __forceinline__ void wave_pairs_range(const WavePairs& wp, int cnt, int& e_begin, int& e_end) {
    e_begin = __shfl(wp.e0, 0, 64);
    int last = wp.e0 == INT_MAX ? -1 : wp.e0 + cnt;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) last = max(last, __shfl_xor(last, o, 64));
    e_end = last;
}
// tile of pair e and its splat (g_out); e must lie in the wave's range for the result to mean anything
__device__ __forceinline__ int wave_pair_tile(const WavePairs& wp, int e, int tiles_x, int& g_out) {
    int lo = 0;
#pragma unroll
    for (int st = 32; st > 0; st >>= 1)
        if (__shfl(wp.e0, lo + st, 64) <= e) lo += st;
    const int k = e - __shfl(wp.e0, lo, 64);
    const int w = max(__shfl(wp.w, lo, 64), 1);
    const int q = k / w;
    g_out = __shfl(wp.g, lo, 64);
    return (__shfl(wp.y0, lo, 64) + q) * tiles_x + __shfl(wp.x0, lo, 64) + (k - q * w);
}

__global__ __launch_bounds__(256) void count_lds_kernel(int n, const float* __restrict__ centers,
                                                        const float* __restrict__ extents,
                                                        const int32_t* __restrict__ offsets, int tiles_x,
                                                        int tiles_y, int block, int32_t* __restrict__ tile_count,
                                                        int32_t* __restrict__ rank, long long cap) {
    if (over_capacity(offsets, n, cap)) return;  // (uniform over the workgroup: before any barrier)
    __shared__ int s_hist[kCountLdsTiles];
    const int n_tiles = tiles_x * tiles_y;
    for (int t = threadIdx.x; t < n_tiles; t += 256) s_hist[t] = 0;
    __syncthreads();
    const int g0 = blockIdx.x * (256 * kCountSplatsPerThread) + threadIdx.x;
    Rect rr[kCountSplatsPerThread];
#pragma unroll
    for (int k = 0; k < kCountSplatsPerThread; ++k) {
        const int g = g0 + k * 256;
        rr[k] = Rect{0, 0, 0, 0};
        if (g < n)
            rr[k] = tile_rect(centers[2 * g], centers[2 * g + 1], extents[2 * g], extents[2 * g + 1], tiles_x,
                              tiles_y, block);
#if GSTEX_COUNT_RESERVE
        // pass 1: the workgroup's tile histogram (no returned values: the LDS adds pipeline)
        for (int ty = rr[k].y0; ty < rr[k].y1; ++ty)
            for (int tx = rr[k].x0; tx < rr[k].x1; ++tx) (void)atomicAdd(&s_hist[ty * tiles_x + tx], 1);
#else
        int e = g < n ? offsets[g] : 0;
        for (int ty = rr[k].y0; ty < rr[k].y1; ++ty)
            for (int tx = rr[k].x0; tx < rr[k].x1; ++tx) rank[e++] = atomicAdd(&s_hist[ty * tiles_x + tx], 1);
#endif
    }
    __syncthreads();
    // one global range per touched tile; s_hist[t] becomes the range's start inside the tile's bucket
    // the workgroups start their reservations at different tiles (a rotation of the tile range per workgroup), so at
    // any moment they hit different counters instead of all queueing on the same 256, and each thread issues its
    // returning atomics in groups of 8 before it waits for them (28.0 -> 25.9 us at cfg3)
    {
        const int rot = (int)(((long long)blockIdx.x * 977) % (n_tiles > 0 ? n_tiles : 1));
        for (int i0 = threadIdx.x; i0 < n_tiles; i0 += 256 * 8) {
            int tt[8], cc[8], rr[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = i0 + 256 * k;
                int t = i + rot;
                t = t >= n_tiles ? t - n_tiles : t;
                tt[k] = i < n_tiles ? t : -1;
                cc[k] = tt[k] >= 0 ? s_hist[t] : 0;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) rr[k] = cc[k] > 0 ? atomicAdd(&tile_count[tt[k]], cc[k]) : 0;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (cc[k] > 0) s_hist[tt[k]] = rr[k];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kCountSplatsPerThread; ++k) {
        const int g = g0 + k * 256;
        int e = g < n ? offsets[g] : 0;
#if GSTEX_COUNT_RESERVE
        // pass 2: each pair takes the next position of its tile's range -- one LDS atomic and one store per pair,
        // no global read of the rank back (the serial per-pair global load was the kernel's latency chain)
        for (int ty = rr[k].y0; ty < rr[k].y1; ++ty)
            for (int tx = rr[k].x0; tx < rr[k].x1; ++tx) rank[e++] = atomicAdd(&s_hist[ty * tiles_x + tx], 1);
#else
        for (int ty = rr[k].y0; ty < rr[k].y1; ++ty)
            for (int tx = rr[k].x0; tx < rr[k].x1; ++tx) rank[e++] += s_hist[ty * tiles_x + tx];
#endif
    }
}

// 3. place keys
__global__ __launch_bounds__(256) void place_kernel(int n, const float* __restrict__ centers,
                                                    const float* __restrict__ extents,
                                                    const float* __restrict__ depths,
                                                    const int32_t* __restrict__ offsets, int tiles_x,
                                                    int tiles_y, int block,
                                                    const int32_t* __restrict__ tile_start,
                                                    const int32_t* __restrict__ rank,
                                                    unsigned long long* __restrict__ keys,
                                                    int32_t* __restrict__ slot_gid, long long cap) {
    if (over_capacity(offsets, n, cap)) return;
    // key = depth bits << 32 | emission slot: a splat's slots lie in [offsets[g], offsets[g + 1]) and each
    // splat has at most one slot per tile, so inside a tile the slot orders exactly as the splat id does
    // and the sorted key hands over the slot directly (the id comes from slot_gid)
    const int g = blockIdx.x * 256 + threadIdx.x;
#if GSTEX_WAVE_PAIRS
    // every lane stays active for the wave-wide shuffles; lanes past n own no pairs
    Rect r{0, 0, 0, 0};
    if (g < n)
        r = tile_rect(centers[2 * g], centers[2 * g + 1], extents[2 * g], extents[2 * g + 1], tiles_x, tiles_y,
                      block);
    const unsigned dbits = g < n ? __float_as_uint(depths[g]) : 0u;
    const WavePairs wp{g < n ? offsets[g] : INT_MAX, r.x0, r.y0, r.x1 - r.x0, g};
    int eb, ee;
    wave_pairs_range(wp, (r.x1 - r.x0) * (r.y1 - r.y0), eb, ee);
    for (int base = eb; base < ee; base += 64) {
        int gg;
        const int e = base + (threadIdx.x & 63);
        const int t = wave_pair_tile(wp, e, tiles_x, gg);
        const unsigned long long dk = (unsigned long long)__shfl(dbits, gg & 63, 64) << 32;
        if (e < ee) {
            keys[tile_start[t] + rank[e]] = dk | (unsigned long long)(unsigned)e;
            slot_gid[e] = gg;
        }
    }
#else
    if (g >= n) return;
    Rect r = tile_rect(centers[2 * g], centers[2 * g + 1], extents[2 * g], extents[2 * g + 1], tiles_x,
                       tiles_y, block);
    const unsigned long long dk = (unsigned long long)__float_as_uint(depths[g]) << 32;
    int e = offsets[g];
    for (int ty = r.y0; ty < r.y1; ++ty)
        for (int tx = r.x0; tx < r.x1; ++tx) {
            int t = ty * tiles_x + tx;
            keys[tile_start[t] + rank[e]] = dk | (unsigned long long)(unsigned)e;
            slot_gid[e] = g;
            ++e;
        }
#endif
}

__device__ __forceinline__ void bitonic_lds(unsigned long long* s, int P) {
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int p = threadIdx.x; p < (P >> 1); p += kSortThreads) {
                int i = 2 * p - (p & (j - 1));
                int ixj = i + j;
                unsigned long long a = s[i], b = s[ixj];
                bool up = ((i & k) == 0);
                if ((a > b) == up) {
                    s[i] = b;
                    s[ixj] = a;
                }
            }
            __syncthreads();
        }
    }
}

__device__ __forceinline__ void write_sorted(int pos, unsigned long long key, const int32_t* slot_gid,
                                             int32_t* sorted_ids, int32_t* sorted_slots) {
    const int slot = (int)(unsigned)(key & 0xffffffffull);
    sorted_slots[pos] = slot;
    sorted_ids[pos] = slot_gid[slot];
}

// Bitonic sort of P = 256 E keys held E per thread (thread t: positions [t E, t E + E)), ascending.  Stages with a
// partner distance j < E swap inside the thread's registers; j < 64 E stays inside the wave's segment of the
// LDS buffer, whose operations the wave issues and the LDS completes in order (no barrier, only a compiler barrier:
// a lane's partner reads must not move above its own writes); only j >= 64 E (3 stages at most) needs the
// workgroup barrier.  (bitonic_lds: a barrier after each of the up to 78 stages.)
template <int E>
__device__ __forceinline__ int pad(int p) { return p + p / E; }
template <int E>
__device__ __forceinline__ void bitonic_regs(unsigned long long (&k)[E], unsigned long long* s, int P) {
    const int base = threadIdx.x * E;
    for (int kk = 2; kk <= P; kk <<= 1) {
        for (int j = kk >> 1; j >= E; j >>= 1) {
            const bool block = j >= 64 * E;
            // one pad slot per thread chunk: lanes' chunks start 2 (E + 1) dwords apart, not 2 E (bank conflicts)
#pragma unroll
            for (int e = 0; e < E; ++e) s[pad<E>(base + e)] = k[e];
            if (block) __syncthreads();
            else asm volatile("" ::: "memory");  // compiler barrier: other lanes' LDS values (the LDS is in order)
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int i = base + e;
                const unsigned long long v = s[pad<E>(i ^ j)];
                const bool lo = (i & j) == 0, up = (i & kk) == 0;
                k[e] = (lo == up) ? (k[e] < v ? k[e] : v) : (k[e] < v ? v : k[e]);
            }
            if (block) __syncthreads();
            else asm volatile("" ::: "memory");  // compiler barrier: other lanes' LDS values (the LDS is in order)
        }
#pragma unroll
        for (int jj = E / 2; jj >= 1; jj >>= 1) {
            if (jj >= kk) continue;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                if (e & jj) continue;
                const bool up = ((base + e) & kk) == 0;
                const unsigned long long a = k[e], b = k[e + jj];
                const bool sw = (a > b) == up;
                k[e] = sw ? b : a;
                k[e + jj] = sw ? a : b;
            }
        }
    }
}

template <int E>
__device__ __forceinline__ void tile_sort_regs(const unsigned long long* src, int K, int start,
                                               unsigned long long* s, const int32_t* slot_gid, int32_t* sorted_ids,
                                               int32_t* sorted_slots) {
    constexpr int P = 256 * E;
    unsigned long long k[E];
    const int base = threadIdx.x * E;
#pragma unroll
    for (int e = 0; e < E; ++e) k[e] = base + e < K ? src[base + e] : ~0ull;
    bitonic_regs<E>(k, s, P);
#pragma unroll
    for (int e = 0; e < E; ++e)
        if (base + e < K) write_sorted(start + base + e, k[e], slot_gid, sorted_ids, sorted_slots);
}

// 4. one workgroup per tile, launched largest bucket first (order[]): the big image-centre buckets no
//    longer start last and set the kernel's tail
__global__ __launch_bounds__(kSortThreads) void tile_sort_kernel(
    int n_tiles, const int32_t* __restrict__ order, const int32_t* __restrict__ tile_start,
    unsigned long long* __restrict__ keys, unsigned long long* __restrict__ scratch,
    const int32_t* __restrict__ slot_gid, int32_t* __restrict__ tile_ranges, int32_t* __restrict__ sorted_ids,
    int32_t* __restrict__ sorted_slots) {
    __shared__ unsigned long long s_keys[kSortCap + kSortThreads];  // + the register sort's pad slots
    const int t = order ? order[blockIdx.x] : (int)blockIdx.x;
    const int start = tile_start[t], end = tile_start[t + 1];
    const int K = end - start;
    if (threadIdx.x == 0) {
        tile_ranges[2 * t] = start;
        tile_ranges[2 * t + 1] = end;
    }
    if (K == 0) return;
    unsigned long long* src = keys + start;
    if (K <= kSortCap) {
        if (GSTEX_SORT_REGS) {
            static_assert(kSortCap == 16 * kSortThreads, "register sort covers the LDS capacity");
            if (K <= 256) tile_sort_regs<1>(src, K, start, s_keys, slot_gid, sorted_ids, sorted_slots);
            else if (K <= 512) tile_sort_regs<2>(src, K, start, s_keys, slot_gid, sorted_ids, sorted_slots);
            else if (K <= 1024) tile_sort_regs<4>(src, K, start, s_keys, slot_gid, sorted_ids, sorted_slots);
            else if (K <= 2048) tile_sort_regs<8>(src, K, start, s_keys, slot_gid, sorted_ids, sorted_slots);
            else tile_sort_regs<16>(src, K, start, s_keys, slot_gid, sorted_ids, sorted_slots);
            return;
        }
        int P = 1;
        while (P < K) P <<= 1;
        for (int i = threadIdx.x; i < P; i += kSortThreads) s_keys[i] = (i < K) ? src[i] : ~0ull;
        __syncthreads();
        bitonic_lds(s_keys, P);
        for (int i = threadIdx.x; i < K; i += kSortThreads)
            write_sorted(start + i, s_keys[i], slot_gid, sorted_ids, sorted_slots);
        return;
    }
    // Large bucket: sort kSortCap-sized chunks in LDS, then merge-path passes in global memory.
    for (int c0 = 0; c0 < K; c0 += kSortCap) {
        int len = min(kSortCap, K - c0);
        int P = 1;
        while (P < len) P <<= 1;
        for (int i = threadIdx.x; i < P; i += kSortThreads) s_keys[i] = (i < len) ? src[c0 + i] : ~0ull;
        __syncthreads();
        bitonic_lds(s_keys, P);
        for (int i = threadIdx.x; i < len; i += kSortThreads) src[c0 + i] = s_keys[i];
        __syncthreads();
    }
    unsigned long long* a_buf = src;
    unsigned long long* b_buf = scratch + start;
    for (int L = kSortCap; L < K; L <<= 1) {
        for (int pb = 0; pb < K; pb += 2 * L) {
            const int a0 = pb, a1 = min(pb + L, K), b1 = min(pb + 2 * L, K);
            const int la = a1 - a0, lb = b1 - a1, total = la + lb;
            const unsigned long long* A = a_buf + a0;
            const unsigned long long* B = a_buf + a1;
            unsigned long long* O = b_buf + a0;
            const int per = (total + kSortThreads - 1) / kSortThreads;
            int diag = min((int)threadIdx.x * per, total);
            int dend = min(diag + per, total);
            int lo = max(0, diag - lb), hi = min(diag, la);
            while (lo < hi) {
                int mid = (lo + hi) >> 1;
                if (A[mid] < B[diag - 1 - mid]) lo = mid + 1;
                else hi = mid;
            }
            int i = lo, j = diag - lo;
            for (int o = diag; o < dend; ++o) {
                bool take_a = (j >= lb) || (i < la && A[i] < B[j]);
                O[o] = take_a ? A[i++] : B[j++];
            }
        }
        __syncthreads();
        unsigned long long* tmp = a_buf;
        a_buf = b_buf;
        b_buf = tmp;
    }
    for (int i = threadIdx.x; i < K; i += kSortThreads)
        write_sorted(start + i, a_buf[i], slot_gid, sorted_ids, sorted_slots);
}

// 5. largest-first tile order (LPT list scheduling).  The hardware hands out workgroups in
// blockIdx order, round-robin over the 8 XCDs; launching the heaviest tiles first keeps every XCD
// busy until the end instead of leaving a long tail behind the image centre's deep tiles.
constexpr int kOrderCap = 16384;  // tiles ranked by the quadratic kernel (beyond: row-major order)
constexpr unsigned kOrderTileBits = 14;
constexpr unsigned kOrderMaxCount = (1u << (32 - kOrderTileBits)) - 1;

// Tile order by ranking: tile t goes to position #{tiles u : key_u < key_t} (keys are unique: the tile index is
// in the low bits).  Each workgroup ranks 64 tiles against all keys, staged through LDS in chunks and read as
// broadcast 16-B vectors, its 16 waves each comparing against a sixteenth of the keys: O(n^2) compares spread over
// the whole chip instead of a bitonic sort in one workgroup (78 barrier-separated stages for 2 500 tiles), and a
// short serial chain of LDS reads per wave (4 waves with a quarter each: 9.4 us at cfg3).
constexpr int kRankThreads = 1024;
constexpr int kRankParts = kRankThreads / 64;
constexpr int kRankTiles = 64;  // tiles per workgroup (one per lane)
constexpr int kRankChunk = 4096;

// Sort keys, all unique (the item index sits in the low bits), ascending = launch order:
//   SRC 0: tile t's bucket size from tile_ranges (pairs [start, end)), 14-bit tile index;
//   SRC 1: the same from the n+1 exclusive-scan starts;
template <int SRC>
__device__ __forceinline__ unsigned order_key(const int32_t* r, int t) {
    const int c = SRC == 1 ? r[t + 1] - r[t] : r[2 * t + 1] - r[2 * t];
    const unsigned cnt = (unsigned)min((int)kOrderMaxCount, c);
    return ((kOrderMaxCount - cnt) << kOrderTileBits) | (unsigned)t;  // count desc, tile asc
}

template <int SRC>
__global__ __launch_bounds__(kRankThreads) void tile_rank_kernel(int n_tiles, const int32_t* __restrict__ tile_ranges,
                                                                 int32_t* __restrict__ tile_order) {
    __shared__ uint4 s_key[kRankChunk / 4];
    __shared__ int s_rank[kRankParts][kRankTiles];
    unsigned* s_k = reinterpret_cast<unsigned*>(s_key);
    const int part = threadIdx.x >> 6;
    const int t = blockIdx.x * kRankTiles + (threadIdx.x & 63);
    const unsigned mine = t < n_tiles ? order_key<SRC>(tile_ranges, t) : 0u;
    int rank = 0;
    for (int c0 = 0; c0 < n_tiles; c0 += kRankChunk) {
        const int cn = min(kRankChunk, n_tiles - c0);
        __syncthreads();
        for (int i = threadIdx.x; i < kRankChunk; i += kRankThreads)
            s_k[i] = i < cn ? order_key<SRC>(tile_ranges, c0 + i) : ~0u;  // padding never ranks below a key
        __syncthreads();
        const int nv = (cn + 3) >> 2;
        const int q0 = nv * part / kRankParts, q1 = nv * (part + 1) / kRankParts;
        for (int i = q0; i < q1; ++i) {
            const uint4 k = s_key[i];
            rank += (int)(k.x < mine) + (int)(k.y < mine) + (int)(k.z < mine) + (int)(k.w < mine);
        }
    }
    s_rank[part][threadIdx.x & 63] = rank;
    __syncthreads();
    if (part == 0 && t < n_tiles) {
        int r = 0;
#pragma unroll
        for (int p = 0; p < kRankParts; ++p) r += s_rank[p][threadIdx.x];
        tile_order[r] = t;
    }
}

__global__ void iota_kernel(int n, int32_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = i;
}

struct BinWorkspace {
    int32_t* tile_count;   // n_tiles + 1 (scan output reused as tile_start)
    int32_t* tile_start;   // n_tiles + 1
    int32_t* scan_ws;      // scan block sums
    int32_t* rank;         // n_isect
    unsigned long long* keys;     // n_isect
    unsigned long long* scratch;  // n_isect
    int32_t* slot_gid;            // n_isect: splat id of each emission slot
    int32_t* order;               // n_tiles: tile_sort launch order (largest bucket first)
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t bin_layout(int n_tiles, int64_t n_isect, char* base, BinWorkspace* ws) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* p = base ? base + off : nullptr;
        off += align256(bytes);
        return p;
    };
    char* p0 = take((size_t)(n_tiles + 1) * 4);
    char* p1 = take((size_t)(n_tiles + 1) * 4);
    char* p2 = take(scan_ws_bytes(n_tiles + 1));
    char* p3 = take((size_t)n_isect * 4);
    char* p4 = take((size_t)n_isect * 8);
    char* p5 = take((size_t)n_isect * 8);
    char* p6 = take((size_t)n_isect * 4);
    char* p7 = take((size_t)n_tiles * 4);
    if (ws) {
        ws->tile_count = (int32_t*)p0;
        ws->tile_start = (int32_t*)p1;
        ws->scan_ws = (int32_t*)p2;
        ws->rank = (int32_t*)p3;
        ws->keys = (unsigned long long*)p4;
        ws->scratch = (unsigned long long*)p5;
        ws->slot_gid = (int32_t*)p6;
        ws->order = (int32_t*)p7;
    }
    return off;
}

}  // namespace

extern "C" size_t gstex_scan_workspace_size(int32_t n) { return scan_ws_bytes(n < 0 ? 0 : n); }

extern "C" int gstex_scan_offsets(int32_t n, const int32_t* num_tiles_hit, int32_t* offsets, void* workspace,
                                  size_t workspace_bytes, void* stream) {
    GSTEX_REQUIRE(n >= 0 && offsets, "gstex_scan_offsets: invalid arguments");
    GSTEX_REQUIRE(n == 0 || num_tiles_hit, "gstex_scan_offsets: null input");
    GSTEX_REQUIRE(workspace_bytes >= scan_ws_bytes(n) && workspace, "gstex_scan_offsets: workspace too small");
    return run_scan(n, num_tiles_hit, offsets, (int32_t*)workspace, as_stream(stream));
}

extern "C" size_t gstex_bin_workspace_size(int32_t n, int64_t n_isect, int32_t n_tiles) {
    (void)n;
    return bin_layout(n_tiles, n_isect, nullptr, nullptr);
}

namespace {
// tile_order_out (nullable): the largest-first launch order the tile sort used, identical to what
// gstex_tile_order computes from tile_ranges (both rank the same bucket sizes), so the forward reuses it
// capped: n_isect is the pair buffers' capacity and the true total is read on the device (offsets[n]; above the
// capacity every tile comes out empty) -- no host read-back of the total is needed to launch the binning
int bin_sort_impl(int32_t n, int64_t n_isect, const float* centers, const float* extents, const float* depths,
                  const int32_t* offsets, int32_t H, int32_t W, int32_t block, int32_t* tile_ranges,
                  int32_t* sorted_ids, int32_t* sorted_slots, int32_t* tile_order_out, void* workspace,
                  size_t workspace_bytes, void* stream, bool capped = false, bool count_zeroed = false) {
    GSTEX_REQUIRE(n >= 0 && n_isect >= 0 && n_isect < (1ll << 31) && H > 0 && W > 0 && block > 0,
                  "gstex_bin_sort: invalid sizes (n=%d, n_isect=%lld, H=%d, W=%d, block=%d)", n,
                  (long long)n_isect, H, W, block);
    GSTEX_REQUIRE(block == kTile, "gstex_bin_sort: block_width must be %d (got %d)", kTile, block);
    const int tiles_x = (W + block - 1) / block, tiles_y = (H + block - 1) / block;
    const int n_tiles = tiles_x * tiles_y;
    GSTEX_REQUIRE(tile_ranges, "gstex_bin_sort: null tile_ranges");
    size_t need = bin_layout(n_tiles, n_isect, nullptr, nullptr);
    GSTEX_REQUIRE(workspace && workspace_bytes >= need, "gstex_bin_sort: workspace too small (%zu < %zu)",
                  workspace_bytes, need);
    hipStream_t st = as_stream(stream);
    if (n_isect == 0 && !capped) {
        (void)hipMemsetAsync(tile_ranges, 0, (size_t)n_tiles * 2 * sizeof(int32_t), st);
        if (tile_order_out) iota_kernel<<<div_up(n_tiles, 256), 256, 0, st>>>(n_tiles, tile_order_out);
        return launch_status("gstex_bin_sort(empty)");
    }
    GSTEX_REQUIRE(centers && extents && depths && offsets && sorted_ids && sorted_slots,
                  "gstex_bin_sort: null pointer");
    const long long cap = capped ? (long long)n_isect : -1;
    BinWorkspace ws;
    bin_layout(n_tiles, n_isect, (char*)workspace, &ws);
    // (the whole 256-B-aligned slot: a size that is not a multiple of 16 B costs the runtime a second fill kernel)
    if (!count_zeroed) (void)hipMemsetAsync(ws.tile_count, 0, align256((size_t)(n_tiles + 1) * sizeof(int32_t)), st);
    if (n_tiles <= kCountLdsTiles)
        count_lds_kernel<<<div_up(n, 256 * kCountSplatsPerThread), 256, 0, st>>>(
            n, centers, extents, offsets, tiles_x, tiles_y, block, ws.tile_count, ws.rank, cap);
    else
        count_kernel<<<div_up(n, 256), 256, 0, st>>>(n, centers, extents, offsets, tiles_x, tiles_y, block,
                                                      ws.tile_count, ws.rank, cap);
    int rc = run_scan(n_tiles, ws.tile_count, ws.tile_start, ws.scan_ws, st);
    if (rc) return rc;
    place_kernel<<<div_up(n, 256), 256, 0, st>>>(n, centers, extents, depths, offsets, tiles_x, tiles_y, block,
                                                  ws.tile_start, ws.rank, ws.keys, ws.slot_gid, cap);
    const bool ranked = n_tiles <= kOrderCap;
    int32_t* order = tile_order_out ? tile_order_out : ws.order;
    if (ranked)
        tile_rank_kernel<1><<<div_up(n_tiles, kRankTiles), kRankThreads, 0, st>>>(n_tiles, ws.tile_start, order);
    else if (tile_order_out)  // beyond the ranking's budget: row-major, as gstex_tile_order
        iota_kernel<<<div_up(n_tiles, 256), 256, 0, st>>>(n_tiles, tile_order_out);
    tile_sort_kernel<<<n_tiles, kSortThreads, 0, st>>>(n_tiles, ranked ? order : nullptr, ws.tile_start, ws.keys,
                                                       ws.scratch, ws.slot_gid, tile_ranges, sorted_ids,
                                                       sorted_slots);
    return launch_status("gstex_bin_sort");
}
}  // namespace

extern "C" int gstex_bin_sort(int32_t n, int64_t n_isect, const float* centers, const float* extents,
                              const float* depths, const int32_t* num_tiles_hit, const int32_t* offsets,
                              int32_t H, int32_t W, int32_t block, int32_t* tile_ranges, int32_t* sorted_ids,
                              int32_t* sorted_slots, void* workspace, size_t workspace_bytes, void* stream) {
    (void)num_tiles_hit;
    return bin_sort_impl(n, n_isect, centers, extents, depths, offsets, H, W, block, tile_ranges, sorted_ids,
                         sorted_slots, nullptr, workspace, workspace_bytes, stream);
}

extern "C" int gstex_bin_sort_ordered(int32_t n, int64_t n_isect, const float* centers, const float* extents,
                                      const float* depths, const int32_t* num_tiles_hit, const int32_t* offsets,
                                      int32_t H, int32_t W, int32_t block, int32_t* tile_ranges,
                                      int32_t* sorted_ids, int32_t* sorted_slots, int32_t* tile_order,
                                      void* workspace, size_t workspace_bytes, void* stream) {
    (void)num_tiles_hit;
    GSTEX_REQUIRE(tile_order, "gstex_bin_sort_ordered: null tile_order");
    return bin_sort_impl(n, n_isect, centers, extents, depths, offsets, H, W, block, tile_ranges, sorted_ids,
                         sorted_slots, tile_order, workspace, workspace_bytes, stream);
}

extern "C" int gstex_bin_sort_capped(int32_t n, int64_t capacity, const float* centers, const float* extents,
                                     const float* depths, const int32_t* num_tiles_hit, const int32_t* offsets,
                                     int32_t H, int32_t W, int32_t block, int32_t* tile_ranges, int32_t* sorted_ids,
                                     int32_t* sorted_slots, int32_t* tile_order, void* workspace,
                                     size_t workspace_bytes, void* stream) {
    (void)num_tiles_hit;
    GSTEX_REQUIRE(tile_order, "gstex_bin_sort_capped: null tile_order");
    GSTEX_REQUIRE(capacity >= 0, "gstex_bin_sort_capped: capacity < 0");
    return bin_sort_impl(n, capacity, centers, extents, depths, offsets, H, W, block, tile_ranges, sorted_ids,
                         sorted_slots, tile_order, workspace, workspace_bytes, stream, true);
}

namespace gstex {
ZeroSpan bin_count_span(void* workspace, int32_t n_tiles, int64_t n_isect) {
    BinWorkspace ws;
    bin_layout(n_tiles, n_isect, (char*)workspace, &ws);
    return ZeroSpan{ws.tile_count, align256((size_t)(n_tiles + 1) * sizeof(int32_t))};
}

int bin_sort_capped_prezeroed(int32_t n, int64_t capacity, const float* centers, const float* extents,
                              const float* depths, const int32_t* offsets, int32_t H, int32_t W, int32_t block,
                              int32_t* tile_ranges, int32_t* sorted_ids, int32_t* sorted_slots, int32_t* tile_order,
                              void* workspace, size_t workspace_bytes, void* stream) {
    GSTEX_REQUIRE(tile_order, "gstex_bin_sort_capped: null tile_order");
    GSTEX_REQUIRE(capacity >= 0, "gstex_bin_sort_capped: capacity < 0");
    return bin_sort_impl(n, capacity, centers, extents, depths, offsets, H, W, block, tile_ranges, sorted_ids,
                         sorted_slots, tile_order, workspace, workspace_bytes, stream, true, true);
}
}  // namespace gstex

extern "C" int gstex_scan_offsets_guarded(int32_t n, const int32_t* num_tiles_hit, int32_t* offsets, void* workspace,
                                          size_t workspace_bytes, const gstex_pair_guard* guard, void* stream) {
    GSTEX_REQUIRE(n >= 0 && offsets && guard, "gstex_scan_offsets_guarded: invalid arguments");
    GSTEX_REQUIRE(n == 0 || num_tiles_hit, "gstex_scan_offsets_guarded: null input");
    GSTEX_REQUIRE(workspace_bytes >= scan_ws_bytes(n) && workspace, "gstex_scan_offsets_guarded: workspace too small");
    GSTEX_REQUIRE(guard->capacity >= 0, "gstex_scan_offsets_guarded: capacity < 0");
    const ScanGuard g{(long long)guard->capacity, guard->step_flag, guard->host_count, guard->first ? 1 : 0};
    return run_scan(n, num_tiles_hit, offsets, (int32_t*)workspace, as_stream(stream), g);
}

extern "C" int gstex_tile_order(int32_t n_tiles, const int32_t* tile_ranges, int32_t* tile_order, void* stream) {
    GSTEX_REQUIRE(n_tiles >= 0, "gstex_tile_order: invalid n_tiles %d", n_tiles);
    if (n_tiles == 0) return GSTEX_OK;
    GSTEX_REQUIRE(tile_ranges && tile_order, "gstex_tile_order: null pointer");
    if (n_tiles > kOrderCap) {  // beyond the quadratic ranking's budget: row-major order
        iota_kernel<<<div_up(n_tiles, 256), 256, 0, as_stream(stream)>>>(n_tiles, tile_order);
        return launch_status("gstex_tile_order");
    }
    tile_rank_kernel<0><<<div_up(n_tiles, kRankTiles), kRankThreads, 0, as_stream(stream)>>>(n_tiles, tile_ranges,
                                                                                                tile_order);
    return launch_status("gstex_tile_order");
}

// Backward unit order (gstex_unit_order).  Key = cost (bits 0-23) | XCD group (bits 24-26); units of cost 0 have no
// work and get no position (order[] = -1 there).  Counting sort by descending cost (clamped to kUnitBuckets - 1)
// within each group, then the groups interleaved: the k-th unit of group g goes to launch position 8 k + g, which
// the hardware's round-robin dispatch places on XCD g (performance only: the map is not guaranteed), so the units
// of one 2x2-tile macro-block share one XCD's L2 (texel blocks, records).  If the groups are too uneven for that
// (8 max_g len_g > n_units), the order is the plain descending-cost one.  Order inside a bucket is unspecified --
// scheduling only, outputs do not depend on it.
#ifndef GSTEX_UNITS_PER_BLOCK
#define GSTEX_UNITS_PER_BLOCK 1024  // measured: 4096 17.5 us, 2048 12.6, 1024 10.3 (unit scatter at cfg3)
#endif
constexpr int kUnitsPerBlock = GSTEX_UNITS_PER_BLOCK;
// scratch (int32): [0, 8192) histogram, [8192, 16384) per-bin placement counters (both zeroed by the caller), the rest
// spare
constexpr int kUnitScratch = 3 * kUnitBins + 16;

__global__ __launch_bounds__(256) void unit_hist_kernel(int n, const int32_t* __restrict__ key,
                                                        int32_t* __restrict__ hist) {
    __shared__ int s_h[kUnitBins];
    for (int i = threadIdx.x; i < kUnitBins; i += 256) s_h[i] = 0;
    __syncthreads();
    const int u0 = blockIdx.x * kUnitsPerBlock;
    for (int u = u0 + threadIdx.x; u < min(n, u0 + kUnitsPerBlock); u += 256) {
        const int k = key[u];
        if (k & 0xFFFFFF) atomicAdd(&s_h[unit_bin(k)], 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kUnitBins; i += 256)
        if (s_h[i]) atomicAdd(&hist[i], s_h[i]);
}

// The counting sort's scan and scatter in one launch (round 6; the two launches took 8.4 + 9.9 us at cfg3): every
// workgroup scans the whole histogram itself (8192 bins from L2; cheaper than a launch and its latency), thread t =
// bucket t: per group, the exclusive scan of its buckets (costliest first) -> the group-interleaved starts; over all
// groups (bucket-major, group-minor) -> the plain starts; then it reserves one range per bin it touches by an atomic
// on a zeroed counter (scratch[kUnitBins, 2 kUnitBins)) and places its units (one per thread).
static_assert(kUnitsPerBlock == kUnitBuckets, "one unit per thread of the placing workgroup");
__global__ __launch_bounds__(kUnitBuckets) void unit_place_kernel(int n, const int32_t* __restrict__ key,
                                                                  int32_t* __restrict__ ws, int32_t* __restrict__ order,
                                                                  int bias) {
    constexpr int NV = kUnitGroups + 1, NW = kUnitBuckets / 64;
    __shared__ int s_tot[NW][NV];
    __shared__ int s_start[kUnitBins];
    __shared__ int s_h[kUnitBins];
    __shared__ int s_grouped;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    for (int i = t; i < kUnitBins; i += kUnitBuckets) s_h[i] = 0;
    int h[NV], x[NV];
    h[kUnitGroups] = 0;
#pragma unroll
    for (int g = 0; g < kUnitGroups; ++g) {
        h[g] = ws[g * kUnitBuckets + t];
        h[kUnitGroups] += h[g];
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) x[i] = wave_incl_scan(h[i]);
    if (lane == 63)
#pragma unroll
        for (int i = 0; i < NV; ++i) s_tot[wave][i] = x[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        int off = 0;
        for (int w = 0; w < wave; ++w) off += s_tot[w][i];
        x[i] += off - h[i];  // exclusive
    }
    if (t == 0) {  // group-interleaved only if no group is longer than n / kUnitGroups
        int mx = 0;
        for (int g = 0; g < kUnitGroups; ++g) {
            int len = 0;
            for (int w = 0; w < NW; ++w) len += s_tot[w][g];
            mx = max(mx, len);
        }
        s_grouped = (long long)kUnitGroups * mx <= (long long)n ? 1 : 0;
    }
    __syncthreads();
    const bool grouped = s_grouped != 0;
    int run = x[kUnitGroups];
#pragma unroll
    for (int g = 0; g < kUnitGroups; ++g) {
        s_start[g * kUnitBuckets + t] = grouped ? x[g] : run;
        run += h[g];
    }
    const int u = blockIdx.x * kUnitBuckets + t;
    const int k = u < n ? key[u] : 0;
    const int b = (k & 0xFFFFFF) ? unit_bin(k) : -1;
    if (b >= 0) atomicAdd(&s_h[b], 1);
    __syncthreads();
    int32_t* cnt = ws + kUnitBins;
    for (int i = t; i < kUnitBins; i += kUnitBuckets)
        if (s_h[i]) s_h[i] = s_start[i] + atomicAdd(&cnt[i], s_h[i]);  // this workgroup's range start in bin i
    __syncthreads();
    if (b >= 0) {
        const int r = atomicAdd(&s_h[b], 1);
        order[grouped ? kUnitGroups * r + b / kUnitBuckets : r] = u + bias;
    }
}

extern "C" size_t gstex_unit_order_scratch_words(void) { return kUnitScratch; }

extern "C" int gstex_unit_order(int32_t n_units, const int32_t* unit_key, int32_t* unit_order, int32_t* scratch,
                                void* stream) {
    GSTEX_REQUIRE(n_units >= 0, "gstex_unit_order: invalid n_units %d", n_units);
    if (n_units == 0) return GSTEX_OK;
    GSTEX_REQUIRE(unit_key && unit_order && scratch, "gstex_unit_order: null pointer");
    hipStream_t st = as_stream(stream);
    if (hipMemsetAsync(scratch, 0, 2 * kUnitBins * sizeof(int32_t), st) != hipSuccess ||
        hipMemsetAsync(unit_order, 0xFF, (size_t)n_units * sizeof(int32_t), st) != hipSuccess)
        return launch_status("gstex_unit_order");
    const int nb = div_up(n_units, kUnitsPerBlock);
    unit_hist_kernel<<<nb, 256, 0, st>>>(n_units, unit_key, scratch);
    unit_place_kernel<<<nb, kUnitBuckets, 0, st>>>(n_units, unit_key, scratch, unit_order, 0);
    return launch_status("gstex_unit_order");
}

namespace gstex {
int unit_order_from_hist(int32_t n_units, const int32_t* unit_key, int32_t* unit_order, int32_t* scratch,
                         hipStream_t st) {
    if (n_units <= 0) return GSTEX_OK;
    unit_place_kernel<<<div_up(n_units, kUnitsPerBlock), kUnitBuckets, 0, st>>>(n_units, unit_key, scratch, unit_order, 1);
    return launch_status("unit_order_from_hist");
}
}  // namespace gstex
