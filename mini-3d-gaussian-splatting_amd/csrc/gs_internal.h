// gs_internal.h -- shared by the library's .hip files; not part of the C ABI.
#pragma once
#include "gsplat_mi355x.h"

// entries per radix sort block (gsplat_mi355x.hip kSortChunk): the row length
// of the sort's digit-count table is div_up(n, kSortBlockEntries)
#ifndef GS_SORT_IPT
#define GS_SORT_IPT 8
#endif
constexpr int32_t kSortBlockEntries = 256 * GS_SORT_IPT;

// set gs_last_error() (fmt has one %s, filled with `what`) and return s
__attribute__((visibility("hidden"))) gs_status gs_internal_fail(gs_status s, const char *fmt, const char *what);
// GS_ERR_LAUNCH with the HIP error text if the last launch failed, else GS_OK
__attribute__((visibility("hidden"))) gs_status gs_internal_check_launch(const char *what);

// gs_radix_sort_pairs; first_counts_ready: the first pass's digit counts are
// in the workspace already (gs_internal_bin_emit_hist built them)
__attribute__((visibility("hidden"))) gs_status gs_internal_radix_sort_pairs(
    uint32_t *keys, uint32_t *vals, uint32_t *keys_alt, uint32_t *vals_alt, int32_t n, int32_t begin_bit,
    int32_t end_bit, int32_t vals_are_iota, void *workspace, size_t workspace_bytes, int32_t *result_in_alt,
    int32_t first_counts_ready, const uint32_t *n_dev, gs_stream_t stream);
// the digit width of gs_radix_sort_pairs' first pass over bits [begin_bit, end_bit)
__attribute__((visibility("hidden"))) int32_t gs_internal_first_pass_bits(int32_t begin_bit, int32_t end_bit);
// gs_bin_count, also clearing the tile sort's first-pass count table of a
// capacity's sort blocks (tile_counts: that sort's workspace; NULL: none)
__attribute__((visibility("hidden"))) gs_status gs_internal_bin_count_hist(const gs_bin_args *a,
                                                                          uint32_t *tile_counts, int32_t bits,
                                                                          gs_stream_t stream);
// gs_bin_emit, also counting the written keys' first-pass digits (width
// bits, shift 0) per sort block into the cleared table
__attribute__((visibility("hidden"))) gs_status gs_internal_bin_emit_hist(const gs_bin_args *a,
                                                                         uint32_t *tile_counts, int32_t bits,
                                                                         gs_stream_t stream);
// A stable sort of n <= gs_internal_small_sort_max() (key, value) pairs by the
// keys' low `bits` bits in one workgroup (LDS passes): keys / vals in
// (vals NULL: the input positions), keys_out / vals_out out -- the result of
// gs_radix_sort_pairs over bits [0, bits) in one launch.
__attribute__((visibility("hidden"))) int32_t gs_internal_small_sort_max(void);
__attribute__((visibility("hidden"))) gs_status gs_internal_small_sort(const uint32_t *keys, const uint32_t *vals,
                                                                      uint32_t *keys_out, uint32_t *vals_out,
                                                                      int32_t n, int32_t bits, const uint32_t *n_dev,
                                                                      gs_stream_t stream);
