// gstex_internal.h — host-side hooks between the library's translation units (not part of the C ABI): the spans the
// training prologue (trainstep.hip) zeroes inside its scan kernel so that the binning and the raster forward launched
// right after it skip their own fill launches.
#pragma once

#include <cstddef>
#include <cstdint>

namespace gstex {

struct ZeroSpan {
    void* ptr;
    size_t bytes;  // a multiple of 16; ptr 16-byte aligned
};

// binning.hip: the per-tile pair counters of a gstex_bin_sort_capped workspace (zeroed before its count kernel)
ZeroSpan bin_count_span(void* workspace, int32_t n_tiles, int64_t n_isect);
// gstex_bin_sort_capped with that span already zeroed on the stream (no fill launch)
int bin_sort_capped_prezeroed(int32_t n, int64_t capacity, const float* centers, const float* extents,
                              const float* depths, const int32_t* offsets, int32_t H, int32_t W, int32_t block,
                              int32_t* tile_ranges, int32_t* sorted_ids, int32_t* sorted_slots, int32_t* tile_order,
                              void* workspace, size_t workspace_bytes, void* stream);
// raster.hip: the span of a raster aux buffer the forward accumulates unit costs, launch order and the unit-order
// histogram into (zeroed before the forward; GSTEX_SETTING_AUX_ZEROED tells the forward it already is)
ZeroSpan raster_aux_zero_span(void* aux, int64_t n_isect, int32_t n_tiles, int32_t channels);

}  // namespace gstex
