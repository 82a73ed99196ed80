// gs_render.hip -- one-call frame orchestration (include/gsplat_mi355x.h,
// "Frame entry points"): gs_render_forward / gs_render_backward run the
// stage entry points of gsplat_mi355x.hip in the order GaussianRenderer.render
// (renderer.py:31-114) and its autograd backward need, inside the library,
// over two caller-owned workspaces laid out here.  A frame then costs the
// host one call per direction (plus the projection backward's), where the
// Python host issued ~15 library calls and ~20 allocations per frame: the
// small configurations (C1, C2) and the trainer were bound by that host time.
// Host code only: every kernel is launched through the stage entry points.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdint.h>
#include <string.h>

#include <stdio.h>

#include <chrono>

#include "gs_internal.h"
#include "gsplat_mi355x.h"

#ifndef GS_EMIT_TILE_HIST
#define GS_EMIT_TILE_HIST 0
#endif

namespace {

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// frame_ws: per-Gaussian and per-pixel buffers (offsets in bytes)
struct FrameLayout {
  size_t records, rects, keys, vals, key_minmax, counters, sort_ws, bin_ws, pair_offset, ranges, pix_flags,
      cell_neval, grad_sums, total;
};

FrameLayout frame_layout(int32_t n, int32_t W, int32_t H, int32_t tiles, int32_t cells) {
  FrameLayout L;
  const size_t un = (size_t)(n > 0 ? n : 0), hw = (size_t)W * (size_t)H;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += al256(bytes);
    return at;
  };
  L.records = take(un * GS_RECORD_FLOATS * 4);
  L.rects = take(un * 8);
  L.keys = take(un * 8);  // [2, n] ping-pong
  L.vals = take(un * 8);
  L.key_minmax = take(8 * ((un + 255) / 256 + 1));
  L.counters = take(4 * GS_NUM_COUNTERS);
  L.sort_ws = take(gs_radix_sort_workspace_bytes(n > 0 ? n : 1));
  L.bin_ws = take(gs_bin_workspace_bytes(n > 0 ? n : 1));
  L.pair_offset = take(un * 4);
  L.ranges = take((size_t)tiles * 8);
  L.pix_flags = take(hw);
  L.cell_neval = take((size_t)tiles * (size_t)(cells > 0 ? cells : 0) * 4);
  L.grad_sums = take(un * GS_PAIR_GRAD_FLOATS * 4);
  L.total = o;
  return L;
}

// tile_ws: per-list-entry buffers for `cap` entries
struct TileLayout {
  size_t tk[2], tv[2], sort_ws, live, flags, total;
  size_t live_words;
};

TileLayout tile_layout(int64_t cap, int32_t tiles, int32_t live_cells, int32_t flag_groups) {
  TileLayout L;
  const size_t uc = (size_t)(cap > 0 ? cap : 0);
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += al256(bytes);
    return at;
  };
  L.tk[0] = take(uc * 4);
  L.tk[1] = take(uc * 4);
  L.tv[0] = take(uc * 4);
  L.tv[1] = take(uc * 4);
  L.sort_ws = take(gs_radix_sort_workspace_bytes((int32_t)(cap > 0 ? cap : 1)));
  L.live_words = live_cells > 0 ? gs_blend_live_words((int32_t)uc, tiles) : 0;
  L.live = take((size_t)(live_cells > 0 ? live_cells : 0) * L.live_words * 8);
  L.flags = take(uc * (size_t)(flag_groups > 0 ? flag_groups : 0));
  L.total = o;
  return L;
}

int32_t div_up_i(int32_t a, int32_t b) { return (a + b - 1) / b; }

bool fb_ok(const gs_frame_buffers &fb, int32_t n, int32_t W, int32_t H, int32_t tiles, int32_t cells,
           size_t *need_frame) {
  const FrameLayout F = frame_layout(n, W, H, tiles, cells);
  *need_frame = F.total;
  return fb.frame_ws && fb.frame_ws_bytes >= F.total;
}

// the visible depth bits fit the window the depth keys were cut to
// (gs_project_args.key_base / key_bits; rasterizer.window_holds)
bool window_holds(uint32_t key_base, int32_t key_bits, uint32_t zmin, uint32_t zmax) {
  if (key_bits >= 32 || zmin > zmax) return true;
  const uint64_t full = (1ull << key_bits) - 1ull;
  const uint64_t lim = key_bits >= 9 ? (full < (255ull << (key_bits - 8)) ? full : (255ull << (key_bits - 8))) : full;
  return zmin >= key_base && (uint64_t)(zmax - key_base) < lim;
}

// An event record on `stream`; inside a stream capture it becomes an event
// record node of the graph (hipEventRecordExternal), so that every replay
// records it -- the timing events of a replayed step.
thread_local char g_event_err[256];
hipError_t record_event(hipEvent_t ev, gs_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t *deps = nullptr;
  size_t ndeps = 0;
  hipError_t e = hipStreamGetCaptureInfo_v2(s, &cs, nullptr, &graph, &deps, &ndeps);
  if (e != hipSuccess) {
    snprintf(g_event_err, sizeof(g_event_err), "%%s: hipStreamGetCaptureInfo_v2: %s", hipGetErrorString(e));
    return e;
  }
  if (cs != hipStreamCaptureStatusActive) {
    e = hipEventRecord(ev, s);
    if (e != hipSuccess) snprintf(g_event_err, sizeof(g_event_err), "%%s: hipEventRecord: %s", hipGetErrorString(e));
    return e;
  }
  // an event record node behind the capture's current frontier, which it
  // then becomes (the documented way to add a node to a stream capture)
  hipGraphNode_t node = nullptr;
  e = hipGraphAddEventRecordNode(&node, graph, deps, ndeps, ev);
  if (e == hipSuccess) e = hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies);
  if (e != hipSuccess) snprintf(g_event_err, sizeof(g_event_err), "%%s: event record node: %s", hipGetErrorString(e));
  return e;
}

}  // namespace

extern "C" {

size_t gs_frame_workspace_bytes(int32_t n, int32_t width, int32_t height, int32_t tile_size) {
  if (n < 0 || width <= 0 || height <= 0 || tile_size < 1) return 0;
  const int32_t tiles = div_up_i(width, tile_size) * div_up_i(height, tile_size);
  return frame_layout(n, width, height, tiles, gs_tile_quads(tile_size)).total;
}

size_t gs_tile_workspace_bytes(int64_t capacity, int32_t num_tiles, int32_t live_cells, int32_t flag_groups) {
  if (capacity < 0 || capacity > 0x7fffffffLL || num_tiles < 0 || live_cells < 0 || flag_groups < 0) return 0;
  return tile_layout(capacity, num_tiles, live_cells, flag_groups).total;
}

gs_status gs_render_forward(gs_render_fwd_args *a, gs_stream_t stream) {
  static const char *what = "gs_render_forward";
  if (!a) return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null args", what);
  const int32_t n = a->g.n, W = a->cam.image_width, H = a->cam.image_height, L = a->cam.tile_size;
  if (n < 0 || W <= 0 || H <= 0 || L < 1) return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: bad sizes", what);
  const int32_t tiles_x = div_up_i(W, L), tiles_y = div_up_i(H, L), tiles = tiles_x * tiles_y;
  const int32_t cells = gs_tile_quads(L);
  size_t need = 0;
  if (!fb_ok(a->fb, n, W, H, tiles, cells, &need))
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: frame workspace missing or below gs_frame_workspace_bytes", what);
  // device_counts: no host read-back -- the T-dependent launches are sized by
  // the tile workspace's capacity and read T (counters[5]) themselves
  const bool dev = a->device_counts != 0;
  if (dev && (a->fb.capacity <= 0 || a->resume))
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: device_counts needs a tile workspace (capacity > 0), no resume",
                            what);
  if (dev && a->fb.flag_groups > 0 && a->fb.flag_groups < cells)
    return gs_internal_fail(GS_ERR_UNSUPPORTED, "%s: device_counts renders tiles of one backward batch only", what);
  if (!dev && (!a->host_counters_dev || !a->host_counters_host))
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: the pinned counter buffer (device and host address) is required",
                            what);
  const FrameLayout F = frame_layout(n, W, H, tiles, cells);
  char *fw = reinterpret_cast<char *>(a->fb.frame_ws);
  float *records = reinterpret_cast<float *>(fw + F.records);
  uint32_t *rects = reinterpret_cast<uint32_t *>(fw + F.rects);
  uint32_t *keys = reinterpret_cast<uint32_t *>(fw + F.keys), *vals = reinterpret_cast<uint32_t *>(fw + F.vals);
  uint32_t *key_minmax = reinterpret_cast<uint32_t *>(fw + F.key_minmax);
  uint32_t *counters = reinterpret_cast<uint32_t *>(fw + F.counters);
  uint32_t *pair_offset = reinterpret_cast<uint32_t *>(fw + F.pair_offset);
  uint32_t *ranges = reinterpret_cast<uint32_t *>(fw + F.ranges);
  gs_status st;
  const size_t un = (size_t)n;
  gs_bin_args ba;
  memset(&ba, 0, sizeof(ba));
  ba.n = n;
  ba.tiles_x = tiles_x;
  ba.tiles_y = tiles_y;
  ba.rects = rects;
  ba.vis = a->vis;
  ba.counters = counters;
  ba.key_minmax = key_minmax;
  ba.workspace = fw + F.bin_ws;
  ba.workspace_bytes = gs_bin_workspace_bytes(n > 0 ? n : 1);
  ba.pair_offset = pair_offset;
  ba.records = records;
  ba.key_base = a->key_base;
  ba.key_bits = a->key_bits;
  ba.step_flags = a->step_flags;
  ba.frame_seq = a->frame_seq;
  ba.device_counts = dev ? 1 : 0;
  if (!a->resume) {
    a->M = a->T = 0;
    a->depth_min_bits = 0xFFFFFFFFu;
    a->depth_max_bits = 0u;
    gs_project_args pa;
    memset(&pa, 0, sizeof(pa));
    pa.cam = a->cam;
    pa.g = a->g;
    pa.means2d = a->means2d;
    pa.conics = a->conics;
    pa.radii = a->radii;
    pa.vis = a->vis;
    pa.records = records;
    pa.rects = rects;
    pa.depth_keys = keys;
    pa.key_base = a->key_base;
    pa.key_bits = a->key_bits;
    pa.key_minmax = key_minmax;
    if ((st = gs_project_forward(&pa, stream))) return st;
    if (n == 0) return GS_OK;
    int32_t alt = 0;
    // a frame whose keys fit one workgroup sorts them there in one launch
    // (the same stable order as the radix passes it replaces)
    if (n <= gs_internal_small_sort_max()) {
      st = gs_internal_small_sort(keys, nullptr, keys + un, vals + un, n, a->key_bits, nullptr, stream);
      alt = 1;
    } else if (a->depth_sort_msd && a->key_bits >= 9 && a->key_bits <= 31)
      st = gs_depth_sort_msd(keys, vals, keys + un, vals + un, n, a->key_bits, fw + F.sort_ws,
                             gs_radix_sort_workspace_bytes(n), key_minmax + 1, &alt, stream);
    else
      st = gs_radix_sort_pairs(keys, vals, keys + un, vals + un, n, 0, a->key_bits, 1, fw + F.sort_ws,
                               gs_radix_sort_workspace_bytes(n), &alt, stream);
    if (st) return st;
    a->depth_alt = alt;
  }
  ba.sorted_ids = vals + (a->depth_alt ? un : 0);
  if (n == 0) return GS_OK;
  const TileLayout T0 = tile_layout(a->fb.capacity, tiles, a->fb.live_cells, a->fb.flag_groups);
  if (a->fb.capacity > 0 && (!a->fb.tile_ws || a->fb.tile_ws_bytes < T0.total))
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: tile workspace below gs_tile_workspace_bytes(capacity, ...)", what);
  char *tw = reinterpret_cast<char *>(a->fb.tile_ws);
  ba.capacity = a->fb.capacity;
  ba.tile_keys = a->fb.capacity > 0 ? reinterpret_cast<uint32_t *>(tw + T0.tk[0]) : nullptr;
  ba.pair_gauss = a->fb.capacity > 0 ? reinterpret_cast<uint32_t *>(tw + T0.tv[0]) : nullptr;
  // GS_EMIT_TILE_HIST=1 (a variant, off): the tile sort's first-pass digit
  // counts come from the emission (the count clears their table in the tile
  // sort's workspace), one histogram kernel less.  Measured at C3: the
  // emission took 23 -> 36 us against the 5.7 us histogram kernel it saves
  // (DESIGN.md section 4), so the product keeps the separate histogram.
  const int32_t bits = tiles > 1 ? 32 - __builtin_clz((uint32_t)(tiles - 1)) : 1;
  const int32_t bits0 = gs_internal_first_pass_bits(0, bits);
  uint32_t *tile_counts =
      (GS_EMIT_TILE_HIST && a->fb.capacity > 0 && !dev) ? reinterpret_cast<uint32_t *>(tw + T0.sort_ws) : nullptr;
  if (dev) {
    // the count (status and T_eff on the device), the emission into the
    // capacity (skipped by the kernel when T exceeds it), and on: no wait
    ba.host_counters = a->host_counters_dev;
    ba.host_seq = a->host_seq;
    if ((st = gs_bin_count(&ba, stream))) return st;
    if ((st = gs_bin_emit(&ba, stream))) return st;
    a->M = a->T = -1;  // (on the device: counters[0..1], and the pinned buffer's copy)
  } else if (!a->resume) {
    // the counts, then -- with a capacity guess -- the emission, queued before
    // the host reads (M, T) back: its kernel time hides the read-back
    ba.host_counters = a->host_counters_dev;
    ba.host_seq = a->host_seq;
    volatile uint32_t *hc = a->host_counters_host;
    hc[4] = 0u;  // (the previous frame's sequence word)
    if ((st = gs_internal_bin_count_hist(&ba, tile_counts, bits0, stream))) return st;
    if (a->fb.capacity > 0 &&
        (st = tile_counts ? gs_internal_bin_emit_hist(&ba, tile_counts, bits0, stream) : gs_bin_emit(&ba, stream)))
      return st;
    // the one host synchronisation of a frame: poll the sequence word the
    // count writes through the pinned buffer's device address (no event, no copy)
    // After 10 s of polling the stream is synchronised and the word read once
    // more (a healthy stream may hold more than 10 s of work ahead of the
    // count); only a count that has still not arrived then is an error.
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1; hc[4] != a->host_seq; ++i) {
      if ((i & 1023u) == 0) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(a->poll_timeout_ms > 0 ? 0 : 10) +
                                                        std::chrono::milliseconds(a->poll_timeout_ms)) {
          if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
            return gs_internal_fail(GS_ERR_LAUNCH, "%s: hipStreamSynchronize failed while waiting for the counters",
                                    what);
          if (hc[4] != a->host_seq)
            return gs_internal_fail(GS_ERR_LAUNCH, "%s: the frame's counters never reached the host", what);
          break;
        }
        sched_yield();
      }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    a->M = (int32_t)hc[0];
    a->T = (int32_t)hc[1];
    a->depth_min_bits = hc[2];
    a->depth_max_bits = hc[3];
    if (!window_holds(a->key_base, a->key_bits, a->depth_min_bits, a->depth_max_bits))
      return GS_RETRY_FULL_KEYS;  // (sort again with 32-bit keys: not an error)
    if (a->M == 0) return GS_OK;  // (renderer.py:74-83: the caller writes the background image)
    if ((int64_t)a->T > a->fb.capacity) return GS_NEED_CAPACITY;
  } else {
    if ((int64_t)a->T > a->fb.capacity)
      return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: resume needs a capacity of at least T", what);
    if (tile_counts) {
      const size_t words = ((size_t)1 << bits0) * (((size_t)a->fb.capacity + kSortBlockEntries - 1) / kSortBlockEntries);
      if (hipMemsetAsync(tile_counts, 0, 4 * words, (hipStream_t)stream) != hipSuccess)
        return gs_internal_fail(GS_ERR_LAUNCH, "%s: count table memset failed", what);
    }
    if ((st = tile_counts ? gs_internal_bin_emit_hist(&ba, tile_counts, bits0, stream) : gs_bin_emit(&ba, stream)))
      return st;
  }
  // the entries the launches are sized for: T, or the capacity with the
  // kernels reading T_eff (counters[5]: T, 0 for a failed frame) themselves
  const int32_t T = dev ? (int32_t)a->fb.capacity : a->T;
  const uint32_t *t_dev = dev ? counters + 5 : nullptr;
  int32_t talt = 0;
  uint32_t *tk = reinterpret_cast<uint32_t *>(tw + T0.tk[0]), *tk1 = reinterpret_cast<uint32_t *>(tw + T0.tk[1]);
  uint32_t *tv = reinterpret_cast<uint32_t *>(tw + T0.tv[0]), *tv1 = reinterpret_cast<uint32_t *>(tw + T0.tv[1]);
  // (the one-workgroup sort and the radix passes are both stable: one order)
  if (T <= gs_internal_small_sort_max() && !tile_counts) {
    if ((st = gs_internal_small_sort(tk, tv, tk1, tv1, T, bits, t_dev, stream))) return st;
    talt = 1;
  } else if ((st = gs_internal_radix_sort_pairs(tk, tv, tk1, tv1, T, 0, bits, 0, tw + T0.sort_ws,
                                                gs_radix_sort_workspace_bytes((int32_t)a->fb.capacity), &talt,
                                                GS_EMIT_TILE_HIST ? 1 : 0, t_dev, stream))) {
    return st;
  }
  a->tile_alt = talt;
  gs_range_args ra;
  memset(&ra, 0, sizeof(ra));
  ra.num_pairs = T;
  ra.num_tiles = tiles;
  ra.sorted_keys = talt ? tk1 : tk;
  ra.ranges = ranges;
  ra.slot_live = (a->zero_slot_flags && a->fb.flag_groups > 0) ? reinterpret_cast<uint8_t *>(tw + T0.flags) : nullptr;
  ra.cells = a->fb.flag_groups;
  ra.num_pairs_dev = t_dev;
  if ((st = gs_tile_ranges(&ra, stream))) return st;
  gs_blend_fwd_args fa;
  memset(&fa, 0, sizeof(fa));
  fa.cam = a->cam;
  fa.tiles_x = tiles_x;
  fa.tiles_y = tiles_y;
  fa.ranges = ranges;
  fa.sorted_gauss = talt ? tv1 : tv;
  fa.records = records;
  fa.image = a->image;
  fa.alpha = a->alpha;
  fa.depth = a->depth;
  fa.pix_flags = reinterpret_cast<uint8_t *>(fw + F.pix_flags);
  fa.cell_neval = reinterpret_cast<uint32_t *>(fw + F.cell_neval);
  fa.pix_neval = a->pix_neval;
  fa.live_bits = a->fb.live_cells > 0 ? reinterpret_cast<uint64_t *>(tw + T0.live) : nullptr;
  fa.live_words = (int64_t)T0.live_words;
  fa.pair_counts = a->pair_counts;
  fa.num_pairs = T;
  return gs_blend_forward(&fa, stream);
}

gs_status gs_render_backward(gs_render_bwd_args *a, gs_stream_t stream) {
  static const char *what = "gs_render_backward";
  if (!a) return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null args", what);
  const int32_t n = a->g.n, W = a->cam.image_width, H = a->cam.image_height, L = a->cam.tile_size;
  if (n < 0 || W <= 0 || H <= 0 || L < 1) return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: bad sizes", what);
  const int32_t tiles_x = div_up_i(W, L), tiles_y = div_up_i(H, L), tiles = tiles_x * tiles_y;
  const int32_t cells = gs_tile_quads(L), G = a->fb.flag_groups;
  size_t need = 0;
  if (!fb_ok(a->fb, n, W, H, tiles, cells, &need))
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: frame workspace missing or below gs_frame_workspace_bytes", what);
  const FrameLayout F = frame_layout(n, W, H, tiles, cells);
  char *fw = reinterpret_cast<char *>(a->fb.frame_ws);
  float *grad_sums = reinterpret_cast<float *>(fw + F.grad_sums);
  a->grad_sums = grad_sums;
  gs_status st;
  const bool dev = a->device_counts != 0;
  if (dev && (a->fb.capacity <= 0 || G < cells))
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: device_counts needs the forward's capacity and one batch", what);
  // (device-resident: T unknown here -- the blend backward is launched over
  // every tile and reads the ranges T_eff made; a failed frame's emission
  // cleared the rectangles, so its gather reads no slot)
  const bool pixel_grads = (dev || (a->M > 0 && a->T > 0)) && a->g_image;
  const int32_t T = dev ? (int32_t)a->fb.capacity : a->T;
  if (pixel_grads) {
    if (!a->pair_grads || G < 1) return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: pair_grads / flag_groups", what);
    if (!a->image || !a->alpha || !a->depth)
      return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: the forward's image / alpha / depth are required", what);
    const TileLayout T0 = tile_layout(a->fb.capacity, tiles, a->fb.live_cells, G);
    char *tw = reinterpret_cast<char *>(a->fb.tile_ws);
    if (!tw || a->fb.tile_ws_bytes < T0.total)
      return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: tile workspace below gs_tile_workspace_bytes", what);
    uint8_t *flags = reinterpret_cast<uint8_t *>(tw + T0.flags);
    gs_blend_bwd_args b;
    memset(&b, 0, sizeof(b));
    b.cam = a->cam;
    b.tiles_x = tiles_x;
    b.tiles_y = tiles_y;
    b.ranges = reinterpret_cast<const uint32_t *>(fw + F.ranges);
    b.sorted_gauss = reinterpret_cast<const uint32_t *>(tw + (a->tile_alt ? T0.tv[1] : T0.tv[0]));
    b.records = reinterpret_cast<const float *>(fw + F.records);
    b.image = a->image;
    b.alpha = a->alpha;
    b.depth = a->depth;
    b.pix_flags = reinterpret_cast<const uint8_t *>(fw + F.pix_flags);
    b.cell_neval = reinterpret_cast<const uint32_t *>(fw + F.cell_neval);
    b.g_image = a->g_image;
    b.g_alpha = a->g_alpha;
    b.g_depth = a->g_depth;
    b.live_bits = a->fb.live_cells > 0 ? reinterpret_cast<const uint64_t *>(tw + T0.live) : nullptr;
    b.live_words = (int64_t)T0.live_words;
    b.pair_grads = a->pair_grads;
    b.slot_live = flags;
    b.num_pairs = T;
    gs_project_bwd_args ga;
    memset(&ga, 0, sizeof(ga));
    ga.g.n = n;
    ga.vis = a->vis;
    ga.rects = reinterpret_cast<const uint32_t *>(fw + F.rects);
    ga.pair_offset = reinterpret_cast<const uint32_t *>(fw + F.pair_offset);
    ga.pair_grads = a->pair_grads;
    ga.slot_live = flags;
    ga.grad_sums = grad_sums;
    hipEvent_t ev0 = (hipEvent_t)a->blend_events[0], ev1 = (hipEvent_t)a->blend_events[1];
    if (ev0 && record_event(ev0, stream) != hipSuccess)
      return gs_internal_fail(GS_ERR_LAUNCH, g_event_err, what);
    const int32_t one = gs_partial_groups(L);
    if (G >= one || G >= cells) {
      // one batch: every cell (or the tile's combined partials)
      b.cell_begin = 0;
      b.cell_count = 0;
      ga.partial_groups = G;
      if (!a->flags_zeroed && hipMemsetAsync(flags, 0, (size_t)T * (size_t)G, (hipStream_t)stream) != hipSuccess)
        return gs_internal_fail(GS_ERR_LAUNCH, "%s: slot flag memset failed", what);
      if ((st = gs_blend_backward(&b, stream))) return st;
      if (ev1 && record_event(ev1, stream) != hipSuccess)
        return gs_internal_fail(GS_ERR_LAUNCH, g_event_err, what);
      if ((st = gs_gather_partials(&ga, 0, stream))) return st;
    } else {
      // cell batches of G (bounded memory), summed in batch order
      for (int32_t c0 = 0, bi = 0; c0 < cells; c0 += G, ++bi) {
        b.cell_begin = c0;
        b.cell_count = cells - c0 < G ? cells - c0 : G;
        ga.partial_groups = b.cell_count;
        if ((bi || !a->flags_zeroed) &&
            hipMemsetAsync(flags, 0, (size_t)T * (size_t)G, (hipStream_t)stream) != hipSuccess)
          return gs_internal_fail(GS_ERR_LAUNCH, "%s: slot flag memset failed", what);
        if ((st = gs_blend_backward(&b, stream))) return st;
        if ((st = gs_gather_partials(&ga, bi ? 1 : 0, stream))) return st;
      }
      if (ev1 && record_event(ev1, stream) != hipSuccess)  // (batches: gathers included)
        return gs_internal_fail(GS_ERR_LAUNCH, g_event_err, what);
    }
  }
  if (!a->project) return GS_OK;  // (the caller runs gs_project_backward itself, e.g. per row range)
  gs_project_bwd_args pb;
  memset(&pb, 0, sizeof(pb));
  pb.cam = a->cam;
  pb.g = a->g;
  pb.means2d = a->means2d;
  pb.conics = a->conics;
  pb.vis = a->vis;
  pb.rects = reinterpret_cast<const uint32_t *>(fw + F.rects);
  pb.pair_offset = reinterpret_cast<const uint32_t *>(fw + F.pair_offset);
  pb.g_means2d = a->g_means2d;
  pb.g_conics = a->g_conics;
  pb.d_xyz = a->d_xyz;
  pb.d_cov3d = a->d_cov3d;
  pb.d_scaling = a->d_scaling;
  pb.d_rotation = a->d_rotation;
  pb.d_color_logits = a->d_color_logits;
  pb.d_opacity = a->d_opacity;
  pb.d_sh_rest = a->d_sh_rest;
  pb.grad_sums = pixel_grads ? grad_sums : nullptr;  // (the sums are there: no gather here)
  if (a->fused_adam) return gs_project_backward_adam(&pb, a->fused_adam, stream);
  return gs_project_backward(&pb, stream);
}

void gs_frame_offsets(int32_t n, int32_t width, int32_t height, int32_t tile_size, size_t out[14]) {
  if (!out) return;
  const int32_t tiles = (width > 0 && height > 0 && tile_size > 0)
                            ? div_up_i(width, tile_size) * div_up_i(height, tile_size) : 0;
  const FrameLayout F = frame_layout(n, width > 0 ? width : 0, height > 0 ? height : 0, tiles,
                                     tile_size > 0 ? gs_tile_quads(tile_size) : 0);
  const size_t v[14] = {F.records, F.rects,  F.keys,    F.vals,      F.key_minmax, F.counters,  F.sort_ws,
                        F.bin_ws,  F.pair_offset, F.ranges, F.pix_flags, F.cell_neval, F.grad_sums, F.total};
  memcpy(out, v, sizeof(v));
}

void gs_tile_offsets(int64_t capacity, int32_t num_tiles, int32_t live_cells, int32_t flag_groups, size_t out[9]) {
  if (!out) return;
  const TileLayout T = tile_layout(capacity, num_tiles, live_cells, flag_groups);
  const size_t v[9] = {T.tk[0], T.tk[1], T.tv[0], T.tv[1], T.sort_ws, T.live, T.flags, T.total, T.live_words};
  memcpy(out, v, sizeof(v));
}

}  // extern "C"
