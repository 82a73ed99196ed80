/*
 * gsplat_mi355x.h -- C ABI of the MI355X (gfx950) Gaussian-splatting rasterizer.
 *
 * Drop-in boundary for GaussianRenderer.render() of
 * Loveof1ife7/mini-3d-gaussian-splatting (src/core/renderer.py:31-367) and the
 * autograd backward the reference gets from torch.  Every stage of the
 * reference's render pipeline maps to one entry point below; each entry
 * point cites the reference function it replaces.
 *
 * Conventions
 *  - Plain C: raw device pointers, sizes, POD structs.  No torch types.
 *  - Stream ordered: every function enqueues work on `stream` (a hipStream_t
 *    passed as void*) and returns without synchronising.
 *  - Caller owns all memory.  The library never allocates; scratch comes from
 *    caller-provided workspaces whose sizes the *_workspace_bytes() queries
 *    return.
 *  - Errors: every entry point returns a gs_status; gs_last_error() returns a
 *    thread-local message for the last non-OK status on the calling thread.
 *    Nothing aborts or exits.
 *  - Re-entrant: no mutable globals; safe from several host threads on
 *    different streams.
 *  - fp32 throughout (the reference computes in fp32).
 */
#ifndef GSPLAT_MI355X_H
#define GSPLAT_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 21
#define GS_DEFAULT_TILE 16    /* renderer.py:24 tile_size default */
#define GS_MAX_TILE 16384     /* tile_size in [1, GS_MAX_TILE]; the reference accepts any int, and a tile
                                 of at least max(W, H) renders the same as any larger one (one tile
                                 holds the image), so callers clamp to max(W, H): images up to
                                 16384 px on an edge render as one tile (ceil(L/8)^2 <= 4.2 M cells;
                                 the blend launches one 64-lane workgroup per cell of 8 tile slots,
                                 and a launch's work-items stay below 2^32) */
#define GS_QUAD 8             /* pixel cells of 8x8, laid out from each tile's origin: a tile of
                                 edge L holds gs_tile_quads(L) = ceil(L/8)^2 of them (edge cells
                                 clipped to the tile); one 64-lane wave renders one cell */
#define GS_MAX_TILES_AXIS 4096 /* ceil(W/L), ceil(H/L) <= 4096 (12-bit tile coordinates) */
#define GS_MAX_RECT_TILES 256 /* a Gaussian's tile rectangle spans <= 256 tiles in x: holds for
                                 any radius_max when ceil(W/L) <= 256, else needs
                                 ceil((2 floor(radius_max) + 1) / L) + 1 <= 256;
                                 gs_project_forward returns GS_ERR_UNSUPPORTED otherwise */
#define GS_RECORD_FLOATS 12   /* per-Gaussian splat record (3 x float4), see DESIGN.md */
#define GS_PAIR_GRAD_FLOATS 10 /* per (list entry, partial group) gradient partial (gs_partial_groups) */
#define GS_PARTIAL_STRIDE 10   /* floats between partials in pair_grads (dense: 40 B each) */
#define GS_NUM_COUNTERS 8     /* [0] visible M, [1] tile touches T, [2] / [3] min / max fp32 bits of the
                                 visible depths (0xFFFFFFFF / 0 when none; see gs_project_args),
                                 [4] the frame status (GS_FRAME_* bits below), [5] the list entries the
                                 later stages use: T, or 0 when the status is non-zero; [6..7] unused */
/* Frame status bits (gs_bin_count, counters[4]): what a device-resident frame
 * (gs_render_fwd_args.device_counts) could not do on the device.  A frame
 * with a non-zero status is drawn with empty tile lists (memory-safe, not
 * the reference's image) and its caller renders it again on the host path. */
#define GS_FRAME_NEED_CAPACITY 1u /* T > the tile workspace's capacity */
#define GS_FRAME_WINDOW_MISS 2u   /* a visible depth left the depth-key window (or an MSD bucket overflowed) */
#define GS_FRAME_EMPTY 4u         /* M == 0: renderer.py:74-83's background image is the host's */

typedef enum gs_status {
  GS_OK = 0,
  GS_ERR_INVALID_ARG = 1,
  GS_ERR_LAUNCH = 2,
  GS_ERR_UNSUPPORTED = 3,
  /* gs_render_forward only -- not errors, what the caller does next: */
  GS_NEED_CAPACITY = 4,   /* T list entries exceed the tile workspace: grow it and call again with resume = 1 */
  GS_RETRY_FULL_KEYS = 5  /* a visible depth left the depth-key window: render again with key_bits = 32 */
} gs_status;

typedef void *gs_stream_t; /* hipStream_t */

/* Camera + settings as the reference renderer reads them.
 * fx,fy,cx,cy come from camera._width/_height/_FoVx/_FoVy exactly as
 * renderer.py:140-147 computes them (python double, rounded to fp32);
 * view is rows 0..2 of camera.world_view_transform() (renderer.py:150-152,
 * untransposed, column-vector convention). */
typedef struct gs_camera {
  int32_t image_width;   /* RenderSettings.image_width  (renderer.py:60) */
  int32_t image_height;  /* RenderSettings.image_height */
  float fx, fy, cx, cy;
  float view[12];        /* row-major 3x4 [R | t] */
  float radius_min;      /* GaussianRenderer(radius_min=0.01) */
  float radius_max;      /* GaussianRenderer(radius_max=50.0): finite, >= radius_min (see GS_MAX_RECT_TILES) */
  float bg[3];           /* RenderSettings.bg_color */
  int32_t tile_size;     /* GaussianRenderer(tile_size=16): 1..GS_MAX_TILE */
  float campos[3];       /* camera centre in world coordinates, -R^T t; read only when sh_degree > 0 */
} gs_camera;

/* Gaussian inputs (the duck-typed GaussianModel accessors).
 * Covariance: either cov3d ([n,9] row-major, = get_covariance) or the raw
 * parameters scaling ([n,3] log-sigma) + rotation ([n,4] q=[w,x,y,z], not
 * necessarily normalised), from which the kernel builds
 * R(normalize(q)) diag(exp(s)^2) R^T as gaussian_model.py:200-207 does. */
typedef struct gs_gaussians {
  int32_t n;
  const float *xyz;          /* [n, xyz_stride] get_xyz */
  int64_t xyz_stride;        /* floats between rows (3 if contiguous) */
  const float *cov3d;        /* [n,9] or NULL */
  const float *scaling;      /* [n,3] raw, used when cov3d == NULL */
  const float *rotation;     /* [n,4] raw, used when cov3d == NULL */
  const float *color_logits; /* [n, color_stride] get_features[:,0,:] (pre-sigmoid, renderer.py:88-92) */
  int64_t color_stride;
  const float *opacity;      /* [n, opacity_stride] get_opacity.squeeze(1) as given (renderer.py:94) */
  int64_t opacity_stride;
  int32_t opacity_is_logit;  /* 1: opacity holds the model's raw _opacity; the kernels apply
                                get_opacity's sigmoid (gaussian_model.py:119-120) and d_opacity
                                is the gradient w.r.t. the logit */
  /* View-dependent colour (off by default).  The reference
   * renders sigmoid(features[:,0,:]) only (renderer.py:88-92; its
   * MathUtils.spherical_harmonics_eval returns coeffs[:,0], math_utils.py:45-49).
   * sh_degree = 0 is exactly that.  sh_degree = d in 1..3 evaluates the
   * degree-d real SH of the view direction dir = normalize(xyz - campos):
   *   logit_c = color_logits[c] + sum_{k=1}^{(d+1)^2-1} Y_k(dir) sh_rest[k-1][c]
   * (Y_k: the 3DGS basis constants and signs; the DC coefficient stays the
   * raw logit, so degree 0 reduces to the reference), colour = sigmoid(logit). */
  int32_t sh_degree;
  const float *sh_rest;      /* [n, sh_rest_stride] rows holding [15,3] (get_features[:,1:,:]) */
  int64_t sh_rest_stride;
} gs_gaussians;

/* ---- Stage 1: _project_gaussians_3d_to_2d + _frustum_culling ----------
 * Replaces renderer.py:117-200 and :201-220.  One thread per Gaussian.
 * Writes the render() outputs means2d (viewspace_points), conics, radii and
 * visibility_filter, plus the splat record, tile rectangle and depth sort
 * key used by the later stages.  No atomics, no counters: the visible
 * count is produced by gs_bin_count. */
typedef struct gs_project_args {
  gs_camera cam;
  gs_gaussians g;
  float *means2d;       /* [n,2] */
  float *conics;        /* [n,4] = [n,2,2] */
  float *radii;         /* [n]   */
  uint8_t *vis;         /* [n]   torch.bool storage */
  float *records;       /* [n, GS_RECORD_FLOATS] */
  uint32_t *rects;      /* [n,2] packed tile rectangle */
  uint32_t *depth_keys; /* [n]   depth sort keys, see key_base */
  /* Depth keys for the sort of renderer.py:231-237.  Z > 0 for a visible
   * Gaussian, so the fp32 bits of Z order as the depths do: a visible g gets
   * depth_keys[g] = bits(Z) - key_base, a culled one 2^key_bits - 1 (last).
   * key_base = 0, key_bits = 32 is the plain float order.  A caller that
   * knows the visible depth range (counters[2..3] of the previous frame,
   * gs_bin_count) may window it to fewer bits and sort bits [0, key_bits):
   * one radix pass less per 8 bits.  The keys are exact only if every
   * visible bits(Z) - key_base < 2^key_bits - 1, which this frame's
   * counters[2..3] tell after gs_bin_count: otherwise sort again with 32. */
  uint32_t key_base;
  int32_t key_bits;     /* 1..32 */
  uint32_t *key_minmax; /* [2 * ceil(n / 256)] per-block min / max of the visible bits(Z), for
                           gs_bin_count's counters[2..3] */
} gs_project_args;
gs_status gs_project_forward(const gs_project_args *a, gs_stream_t stream);

/* ---- Stage 2 / 4: device LSD radix sort (u32 key, u32 value) -----------
 * Replaces torch.argsort in _sort_gaussians_by_depth (renderer.py:231-237)
 * and the per-tile list build (:277-298).  Stable.  Sorts bits
 * [begin_bit, end_bit) of keys in ceil((end-begin)/8) passes, ping-ponging
 * between (keys, vals) and (keys_alt, vals_alt); *result_in_alt tells the
 * caller which pair holds the result (known on the host without a sync).
 * vals_are_iota != 0: the first pass reads values 0..n-1 instead of vals
 * (vals is still used as ping-pong storage). */
size_t gs_radix_sort_workspace_bytes(int32_t n);
gs_status gs_radix_sort_pairs(uint32_t *keys, uint32_t *vals, uint32_t *keys_alt,
                              uint32_t *vals_alt, int32_t n, int32_t begin_bit,
                              int32_t end_bit, int32_t vals_are_iota, void *workspace,
                              size_t workspace_bytes, int32_t *result_in_alt,
                              gs_stream_t stream);

/* Windowed depth keys (9 <= key_bits <= 32, gs_project_args.key_bits): the
 * same result as gs_radix_sort_pairs(keys, vals, keys_alt, vals_alt, n, 0,
 * key_bits, 1, ...) -- values = input positions, stable -- in one 8-bit MSD
 * pass plus one LDS-resident sort per top-digit bucket (one workgroup each).
 * The result is always in (keys_alt, vals_alt) (*result_in_alt = 1).
 * Preconditions: visible keys < 255 << (key_bits - 8); 2^key_bits - 1 is the
 * culled sentinel (its bucket stays in index order).  A bucket of more than
 * 16384 keys is left unsorted and 0xFFFFFFFF is stored to *overflow_word
 * (renderer: the depth-max word of gs_project_args.key_minmax, so the frame's
 * window check fails and it is sorted again with gs_radix_sort_pairs).
 * The buckets are sorted by the low key_bits - 8 bits in ceil((key_bits - 8)
 * / 8) LDS passes.  Workspace: gs_radix_sort_workspace_bytes(n).  key_bits
 * outside 9..32 returns GS_ERR_UNSUPPORTED. */
gs_status gs_depth_sort_msd(uint32_t *keys, uint32_t *vals, uint32_t *keys_alt, uint32_t *vals_alt,
                            int32_t n, int32_t key_bits, void *workspace, size_t workspace_bytes,
                            uint32_t *overflow_word, int32_t *result_in_alt, gs_stream_t stream);

/* ---- Stage 3: tile binning (renderer.py:263-298) ----------------------
 * gs_bin_count: per-Gaussian tile-touch counts and visibility in depth order,
 *   reduced to per-block partial sums and scanned; the callee zeroes
 *   counters, then counters[0] = M (visible), counters[1] = T (touches).
 *   It also numbers the gradient slots (one per touched tile) in
 *   Gaussian-index order, a Gaussian's slots consecutive: pair_offset is
 *   written here (chunk-local) and completed by gs_bin_emit.
 * gs_bin_emit : one (tile id, Gaussian id) entry per touched tile, emitted in
 *   depth order (so a stable sort by tile keeps depth order inside a tile),
 *   written coalesced; pair_offset[g] = g's first gradient slot, also stored
 *   in the Gaussian's record (word 10) for the backward's slot addressing. */
size_t gs_bin_workspace_bytes(int32_t n);
typedef struct gs_bin_args {
  int32_t n;
  int32_t tiles_x, tiles_y;
  const uint32_t *sorted_ids; /* [n] depth-sorted Gaussian ids (visible first) */
  const uint32_t *rects;      /* [n,2] from gs_project_forward (cleared by gs_bin_emit of a failed
                                 device-resident frame, see device_counts) */
  const uint8_t *vis;         /* [n]   from gs_project_forward */
  uint32_t *counters;         /* [GS_NUM_COUNTERS] */
  const uint32_t *key_minmax; /* gs_project_args.key_minmax (reduced into counters[2..3]) */
  void *workspace;             /* gs_bin_workspace_bytes(n); gs_bin_count leaves the per-block
                                  partials and the depth-ordered rectangles there for gs_bin_emit:
                                  pass the same workspace to both, untouched in between */
  size_t workspace_bytes;
  /* emit outputs (tile_keys / pair_gauss / records ignored by gs_bin_count) */
  uint32_t *tile_keys;   /* [T] */
  uint32_t *pair_gauss;  /* [T] */
  uint32_t *pair_offset; /* [n] indexed by Gaussian id: first gradient slot (both calls write it) */
  float *records;        /* [n, GS_RECORD_FLOATS]: word 10 <- pair_offset bits */
  int64_t capacity;      /* entries tile_keys / pair_gauss hold.  gs_bin_emit does nothing
                            when T = counters[1] > capacity, so it may be queued before T is
                            read back (then emit again into buffers of >= T entries) */
  uint32_t *host_counters; /* optional [8]: the device address of pinned host memory
                              (hipHostGetDevicePointer) that gs_bin_count also writes
                              counters[0..3] to, then -- after a system-scope fence --
                              host_seq to [4]: the caller polls [4] for the value it passed
                              and reads (M, T) with no copy and no event in the stream.
                              NULL: counters only */
  uint32_t host_seq;
  /* The frame status (counters[4], GS_FRAME_*), formed by gs_bin_count from
   * (M, T, the depth range) against capacity and the depth-key window the
   * keys were cut to (gs_project_args.key_base / key_bits): */
  uint32_t key_base;
  int32_t key_bits;        /* 0: no window check */
  uint32_t *step_flags;    /* optional device word: the status is ORed into it (sticky until the caller
                              clears it; gs_adam_args.skip_flag reads it) */
  int32_t device_counts;   /* a device-resident frame (gs_render_fwd_args.device_counts): when the
                              status is non-zero, gs_bin_emit emits nothing and clears every
                              rectangle (rects), so that the frame's backward gathers zero slots --
                              none past the capacity -- and the caller redoes the frame */
  uint32_t *frame_seq;     /* optional device word: incremented by every gs_bin_count; its new value is
                              written to host_counters[4] in place of host_seq (a captured graph
                              replays one frame per value).  host_counters also gets [5] the status,
                              [6] the step flags after this frame (the status without step_flags) and,
                              when this frame is the first to set them, [7] its sequence value */
} gs_bin_args;
gs_status gs_bin_count(const gs_bin_args *a, gs_stream_t stream);
gs_status gs_bin_emit(const gs_bin_args *a, gs_stream_t stream);

/* Per-tile [start,end) ranges of the tile-sorted entries.  Replaces the
 * tile_lists of renderer.py:266 (the sorted values are the Gaussian ids). */
typedef struct gs_range_args {
  int32_t num_pairs;           /* T */
  int32_t num_tiles;
  const uint32_t *sorted_keys; /* [T] tile ids, sorted */
  uint32_t *ranges;            /* [num_tiles,2] */
  uint8_t *slot_live;          /* optional (NULL: none): zeroed here, [T, cells] -- the backward's
                                  gs_blend_bwd_args.slot_live, cleared without a kernel of its own */
  int32_t cells;               /* gs_partial_groups(tile_size), with slot_live */
  const uint32_t *num_pairs_dev; /* optional device word (counters[5]): the entries are
                                  min(*num_pairs_dev, num_pairs), num_pairs only bounding them (a
                                  launch sized by capacity before T is known on the host) */
} gs_range_args;
gs_status gs_tile_ranges(const gs_range_args *a, gs_stream_t stream);

/* ---- Stage 5: _tile_rasterization blend, forward -------------------------
 * renderer.py:273-367: per pixel (integer coordinates) front-to-back alpha
 * compositing of its tile's list, termination once A >= 0.995, background
 * composite (bg counted twice, as the reference does), clamps, depth
 * normalisation.  One 64-lane workgroup per (tile, 8x8 cell), the cells of
 * a tile independent of each other, each walking the tile's list.  What the
 * backward needs beside the outputs themselves: pix_flags (one byte per
 * pixel: which clamps blocked), cell_neval (per cell, the evaluated prefix)
 * and the liveness bitmap. */
typedef struct gs_blend_fwd_args {
  gs_camera cam;
  int32_t tiles_x, tiles_y;
  const uint32_t *ranges;       /* [num_tiles,2] */
  const uint32_t *sorted_gauss; /* [T] */
  const float *records;         /* [n, GS_RECORD_FLOATS] */
  float *image;                 /* [3,H,W] */
  float *alpha;                 /* [H,W]   */
  float *depth;                 /* [H,W]   */
  uint8_t *pix_flags;           /* [H*W] the backward's per-pixel state beside the outputs: bit c
                                   (c = 0..2) set where channel c's composite left [0, 1] (its clamp
                                   blocks the gradient), bit 3 likewise for alpha */
  uint32_t *cell_neval;         /* [num_tiles * gs_tile_quads(tile_size)]: per (tile, 8x8 cell q),
                                   at tile * cells + q, the entries of the tile's list up to the last
                                   one any of the cell's pixels evaluated */
  uint64_t *live_bits;          /* [gs_tile_quads(tile_size), live_words]: see gs_blend_live_words;
                                   NULL: none written (a caller's memory budget for large tiles; the
                                   backward then replays every entry of a cell's evaluated prefix) */
  int64_t live_words;
  uint32_t *pair_counts;        /* [H*W] or NULL: each pixel's contributing pairs (c > 0), the
                                   work counter C of SURVEY 8(d); measurement only */
  int32_t num_pairs;            /* T, the entries of sorted_gauss: tile ranges are clamped to it */
  uint32_t *pix_neval;          /* [H*W] or NULL: each pixel's evaluated entries (the work counter
                                   E of SURVEY 8(d), and the oracle's decision-forced replay);
                                   measurement only */
} gs_blend_fwd_args;
gs_status gs_blend_forward(const gs_blend_fwd_args *a, gs_stream_t stream);

/* Words per cell of the liveness bitmap the forward writes for the
 * backward: bit i of live_bits[q * live_words + ranges[2t] / 64 + t + i / 64]
 * is set iff list entry i of tile t reached (exp(-s/2) >= 1e-5) some
 * still-running pixel of the tile's 8x8 cell q = qx + qy * ceil(L/8)
 * (pixels [qx*8, qx*8+8) x [qy*8, qy*8+8) from the tile's origin) -- the
 * backward replays exactly those (entry, cell) pairs.  Bits past a cell's
 * last evaluated entry are left unwritten. */
size_t gs_blend_live_words(int32_t num_pairs, int32_t num_tiles);
/* Cells per tile: ceil(tile_size / 8)^2 (4 for the default 16); 0 if out of range. */
int32_t gs_tile_quads(int32_t tile_size);
/* Gradient partials a one-batch gs_blend_backward writes per list entry: one
 * per 8x8 cell, gs_tile_quads(tile_size) (4 for the default 16x16 tile); 0 if
 * out of range.  A caller whose [T, cells] partial buffer would not fit its
 * memory budget (large tiles: (L/8)^2 cells) replays the cells in batches
 * (gs_blend_bwd_args.cell_begin / cell_count), summing each batch with
 * gs_gather_partials(accumulate) before the next: bounded memory, the same
 * fixed summation order on every run (deterministic at every tile size). */
int32_t gs_partial_groups(int32_t tile_size);

/* ---- Backward of the blend -------------------------------------------
 * Re-walks each pixel's list front-to-back (bit-identical replay of the
 * forward's decisions) over the entries the forward's liveness bitmap marks
 * for its 8x8 cell, and writes one partial gradient per (entry, partial
 * group): pair_grads[G e + q] = {dmu_x, dmu_y, dQ00, dQ01(=dQ10), dQ11,
 * d_opacity, d_r, d_g, d_b, d_z} summed over group q's pixels, and sets
 * slot_live[G e + q] = 1; G = gs_partial_groups(tile_size), e = the entry's
 * gradient slot (pair_offset[g] + its tile's index in g's rectangle).  One
 * 64-lane workgroup per (tile, cell), and the group is the cell.  Groups
 * that did not replay the entry write nothing.  No atomics: deterministic.
 * A launch replays the cells [cell_begin, cell_begin + cell_count) of every
 * tile (cell_count 0 with cell_begin 0: all of them); G is then cell_count
 * and group q - cell_begin holds cell q's partial. */
typedef struct gs_blend_bwd_args {
  gs_camera cam;
  int32_t tiles_x, tiles_y;
  const uint32_t *ranges;
  const uint32_t *sorted_gauss;
  const float *records;         /* with pair offsets (gs_bin_emit) */
  const float *image;           /* the forward's outputs, unmodified */
  const float *alpha;
  const float *depth;
  const uint8_t *pix_flags;     /* gs_blend_fwd_args.pix_flags / cell_neval of the same forward */
  const uint32_t *cell_neval;
  const float *g_image;         /* [3,H,W] dL/dimage */
  const float *g_alpha;         /* [H,W] or NULL */
  const float *g_depth;         /* [H,W] or NULL */
  const uint64_t *live_bits;    /* the forward's liveness bitmap */
  int64_t live_words;
  float *pair_grads;            /* [T, G, GS_PARTIAL_STRIDE], G = the batch's cell_count */
  uint8_t *slot_live;           /* [T, G], zeroed by the caller (or gs_tile_ranges) */
  int32_t num_pairs;            /* T, the entries of sorted_gauss: tile ranges are clamped to it */
  int32_t cell_begin;           /* the batch's first cell (0) */
  int32_t cell_count;           /* the batch's cells (0: gs_tile_quads(tile_size), the whole tile) */
} gs_blend_bwd_args;
gs_status gs_blend_backward(const gs_blend_bwd_args *a, gs_stream_t stream);
/* Diagnostic (SURVEY 8(d) lane efficiency; not on the render path): the same
 * replay as gs_blend_backward at the default tile (one batch), counting its
 * phase-A lanes.  hist: device [2][65] uint64, added to -- per replayed
 * (entry, cell), [0][r] counts replays entered by r running lanes (lanes of
 * the cell's pixels whose transmittance has not terminated), [1][c] replays
 * where c lanes' pairs contribute (weight > 0).  per_group: device [G][4]
 * uint32 overwritten, G = gs_blend_backward_groups(tiles_x, tiles_y, 4),
 * workgroup b = (tile, cell) per gs_blend_backward's grid: replays, replays
 * entered with >= 32 running lanes, sum of running lanes, sum of
 * contributing lanes (empty workgroups: zeros).  The gradient partials are
 * written as by gs_blend_backward. */
int64_t gs_blend_backward_groups(int32_t tiles_x, int32_t tiles_y, int32_t cell_count);
gs_status gs_blend_backward_lane_stats(const gs_blend_bwd_args *a, uint64_t *hist, uint32_t *per_group,
                                       gs_stream_t stream);

/* ---- Backward of the projection ----------------------------------------
 * Sums each Gaussian's slot partials (slots [pair_offset[g], pair_offset[g]
 * + touches), the groups slot_live flags), adds cotangents on the viewspace_points /
 * conics outputs, and chains through sigmoid(colour), inv(cov2d),
 * J cov_cam J^T, Rv Sigma Rv^T, the perspective Jacobian J(X,Y,Z) and
 * Xc = Rv Xw + Tv (autograd of renderer.py:117-200), and, on the raw path,
 * through Sigma(exp(s), normalize(q)) (gaussian_model.py:200-207), and with
 * sh_degree > 0 through the SH colour into sh_rest and (via the view
 * direction) into xyz. */
typedef struct gs_project_bwd_args {
  gs_camera cam;
  gs_gaussians g;
  const float *means2d, *conics;
  const uint8_t *vis;
  const uint32_t *rects;
  const uint32_t *pair_offset;
  const uint32_t *order;       /* [n] permutation to walk the Gaussians in (the gather and the
                                  projection backward), or NULL: index order (slots are numbered in
                                  index order, so NULL reads them coalesced) */
  const float *pair_grads;     /* [T,G,GS_PARTIAL_STRIDE] (G = partial_groups), summed into grad_sums
                                  first; NULL: no blend gradient (T == 0), or -- with grad_sums --
                                  the sums are already there (gs_gather_partials, cell batches) */
  const float *g_means2d;      /* [n,2] or NULL */
  const float *g_conics;       /* [n,4] or NULL */
  float *d_xyz;                /* [n,3] */
  float *d_cov3d;              /* [n,9]  (cov3d path) */
  float *d_scaling;            /* [n,3]  (raw path)   */
  float *d_rotation;           /* [n,4]  (raw path)   */
  float *d_color_logits;       /* [n,3] */
  float *d_opacity;            /* [n]   */
  float *d_sh_rest;            /* [n,15,3] contiguous, written when g.sh_degree > 0 (zeros past the degree) */
  const uint8_t *slot_live;    /* [T,G] from gs_blend_backward; required with pair_grads */
  float *grad_sums;            /* [n, GS_PAIR_GRAD_FLOATS]: g's partials summed (written first when
                                  pair_grads is given, else read as is); NULL: no blend gradient */
  int32_t partial_groups;      /* G of pair_grads / slot_live: the blend backward's cell_count */
} gs_project_bwd_args;
gs_status gs_project_backward(const gs_project_bwd_args *a, gs_stream_t stream);
/* The gather alone: grad_sums[g] = (accumulate ? grad_sums[g] : 0) + the sum
 * of g's partials in pair_grads / slot_live (partial_groups per slot), for a
 * blend backward run in cell batches: batch b's sums are added after batch
 * b - 1's, a fixed order.  Reads vis, rects, pair_offset, g.n. */
gs_status gs_gather_partials(const gs_project_bwd_args *a, int32_t accumulate, gs_stream_t stream);

/* ---- Adam step over several parameter tensors, one launch -----------------
 * SURVEY 8(f) row 1 (fused Adam), the optimizer the reference builds in
 * src/core/optimizer.py:100-113 (torch.optim.Adam, 5 parameter groups).
 * torch.optim.Adam semantics (amsgrad off, weight_decay 0):
 *   m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2
 *   p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
 * Tensors with grad == NULL are skipped (torch skips params without grad).
 * param_out: NULL updates p in place (torch's behaviour); otherwise p is
 * only read and the updated parameter is written to param_out (same
 * numel, no overlap with p) -- the same reads and writes as the in-place
 * step, e.g. for a benchmark that renders one fixed scene every step. */
#define GS_ADAM_MAX_TENSORS 8
typedef struct gs_adam_tensor {
  float *param, *exp_avg, *exp_avg_sq;
  const float *grad;     /* NULL: skip */
  int64_t numel;
  float lr;
  float bias_correction1; /* 1 - beta1^step */
  float bias_correction2_sqrt; /* sqrt(1 - beta2^step) */
  float *param_out;       /* NULL: in place */
} gs_adam_tensor;
typedef struct gs_adam_args {
  int32_t num_tensors;
  float beta1, beta2, eps;
  gs_adam_tensor t[GS_ADAM_MAX_TENSORS];
  /* Replayed steps (a captured graph whose kernel arguments are fixed):
   * skip_flag: optional device word -- non-zero: the launch updates nothing
   *   (gs_bin_args.step_flags: the frame of this step failed on the device
   *   and the caller redoes the step on the host path);
   * hyper / hyper_row: optional -- tensor i's lr, bias_correction1 and
   *   bias_correction2_sqrt are read from hyper[(r * GS_ADAM_MAX_TENSORS + i)
   *   * 3 + 0..2], r = *hyper_row (a device word, e.g. gs_bin_args.frame_seq),
   *   instead of t[i]; the caller fills the rows the replays will reach. */
  const uint32_t *skip_flag;
  const float *hyper;
  const uint32_t *hyper_row;
} gs_adam_args;
gs_status gs_adam_step(const gs_adam_args *a, gs_stream_t stream);

/* Optimizer in the backward (opt-in; one rank, no gradient hooks): the
 * projection backward of the training configuration (raw scaling / rotation,
 * opacity logit, DC colour, blend sums in grad_sums or pair_grads, no
 * viewspace / conic cotangents) applies the Adam update of gs_adam_step --
 * the same fp32 operations -- to each parameter where its gradient is formed,
 * instead of writing d_* (not read; no gradient reaches HBM).  adam->t[0..4]
 * are xyz, colour logits, opacity logit, scaling, rotation: param = the arrays
 * of a->g (dense rows), their moments, param_out (NULL: in place); grad is
 * ignored.  skip_flag / hyper / hyper_row as in gs_adam_args.  Saves the
 * gradients' write and read and the parameters' second read (~168 B per
 * Gaussian) and a launch.  GS_ERR_UNSUPPORTED outside that configuration. */
gs_status gs_project_backward_adam(const gs_project_bwd_args *a, const gs_adam_args *adam, gs_stream_t stream);

/* ---- Photometric loss ---------------------------------
 * total = (1 - lambda) * L1 + lambda * D-SSIM, the objective of GaussianLoss
 * (src/core/loss.py:41-63): L1 = mean |pred - target| (:56); D-SSIM =
 * 1 - mean(clamp(SSIM map, 0, 1)) over the statistics SSIMLoss builds
 * (:17-39): a K-tap Gaussian window with sigma = K/6, separable, zero
 * padding, C1 = 0.01^2, C2 = 0.03^2.  The reference SSIMLoss.forward ends
 * without a return; its caller consumes the value as `dssim` (:57-58), which
 * is the D-SSIM form implemented here.  Deterministic (fixed-order
 * reductions, no atomics). */
#define GS_LOSS_MAX_WINDOW 11
typedef struct gs_loss_args {
  int32_t channels, height, width; /* pred/target/d_pred: [C,H,W] fp32 contiguous */
  const float *pred, *target;
  float lambda_dssim;                /* loss.py:42 default 0.2 */
  int32_t window;                    /* odd, 1..GS_LOSS_MAX_WINDOW (loss.py:10 default 11) */
  float c1, c2;                      /* loss.py:14-15 */
  void *workspace;                   /* gs_loss_workspace_bytes */
  size_t workspace_bytes;
  float *maps;                       /* [3,C,H,W] written by the forward for the backward, or NULL */
  float *out;                        /* [3] total, l1, dssim (device) */
  const float *g_total;              /* backward: dL/dtotal (device scalar), NULL = 1 */
  float *d_pred;                     /* backward: [C,H,W] */
} gs_loss_args;
size_t gs_loss_workspace_bytes(int32_t channels, int32_t height, int32_t width);
gs_status gs_loss_forward(const gs_loss_args *a, gs_stream_t stream);
gs_status gs_loss_backward(const gs_loss_args *a, gs_stream_t stream);

/* ---- Densification ------------------------------------
 * One pass of split / clone / prune over the model's raw parameters
 * (gaussian_model.py:130-175 density_and_split / density_and_clone,
 * optimizer.py:64-66 opacity prune), with the Adam moments remapped: kept
 * Gaussians carry theirs, new ones start at zero.  Per Gaussian i, on the
 * pre-densify state: g = |dL/dxyz_i|, s = mean(exp(scaling_i));
 *   split = g > grad_threshold and s > split_size * scene_extent (:137):
 *     i is replaced by two children xyz -/+ R(q)[:,0] * 0.5 s, scaling
 *     log(0.75 exp(scaling)), rotation normalize(q), opacity
 *     clamp(logit(sigmoid(op)), -6, 6), features copied (:139-154);
 *   clone = g > grad_threshold and s < clone_size * scene_extent (:166):
 *     i stays and a copy is added at xyz + N(0,1)^3 * 0.5 s (:169-178);
 *   prune: every output whose sigmoid(opacity) <= min_opacity is dropped.
 * Output order: kept originals, split "-" children, split "+" children,
 * clones; each in the original index order.  (The reference cannot run
 * these: _append_points reads a missing `_scaling_log` (:229).)  Two
 * phases: gs_densify_count writes counters, the caller sizes the outputs. */
#define GS_DENSIFY_SPLIT 1
#define GS_DENSIFY_CLONE 2
#define GS_DENSIFY_PRUNE 4
typedef struct gs_model_arrays {
  float *xyz;           /* [n,3]   _xyz */
  float *features_dc;   /* [n,3]   _features_dc */
  float *features_rest; /* [n,rest_floats] _features_rest */
  float *scaling;       /* [n,3]   _scaling (log) */
  float *rotation;      /* [n,4]   _rotation */
  float *opacity;       /* [n]     _opacity (logit) */
} gs_model_arrays;
typedef struct gs_densify_args {
  int32_t n;
  int32_t rest_floats;
  gs_model_arrays in;             /* read only */
  const float *xyz_grad;          /* [n,3], or NULL: nothing is split or cloned */
  float grad_threshold, scene_extent;
  float split_size, clone_size;   /* 0.03, 0.01 (gaussian_model.py:137,166) */
  float min_opacity;              /* 0.01 (optimizer.py:64) */
  int32_t flags;                  /* GS_DENSIFY_SPLIT | _CLONE | _PRUNE */
  uint64_t seed;                  /* clone jitter: counter-based normals, deterministic */
  gs_model_arrays adam_m_in, adam_v_in;   /* NULL members: not remapped */
  void *workspace;
  size_t workspace_bytes;
  uint32_t *counters;             /* [4]: kept, split children per side, clones, n_out */
  gs_model_arrays out, adam_m_out, adam_v_out;
} gs_densify_args;
size_t gs_densify_workspace_bytes(int32_t n);
gs_status gs_densify_count(const gs_densify_args *a, gs_stream_t stream);
gs_status gs_densify_emit(const gs_densify_args *a, gs_stream_t stream);

/* ---- Frame entry points: the stages above in one call per direction -------
 * gs_render_forward runs what GaussianRenderer.render does (renderer.py:31-114)
 * -- projection + culling, depth sort, binning, tile sort, ranges, blend --
 * and gs_render_backward its autograd backward, over two caller-owned
 * workspaces the library lays out: a frame workspace (per Gaussian and per
 * pixel, gs_frame_workspace_bytes) and a tile workspace (per list entry, for up
 * to `capacity` entries, gs_tile_workspace_bytes).  The host reads the
 * frame's counts (M, T, the visible depth range) back once, inside
 * gs_render_forward, by polling a pinned buffer the count writes through its
 * device address.  Both workspaces must stay untouched from the forward to
 * its backward. */
typedef struct gs_frame_buffers {
  void *frame_ws;        /* gs_frame_workspace_bytes(n, W, H, tile_size) */
  size_t frame_ws_bytes;
  void *tile_ws;         /* gs_tile_workspace_bytes(capacity, tiles, live_cells, flag_groups) */
  size_t tile_ws_bytes;
  int64_t capacity;      /* list entries the tile workspace holds */
  int32_t live_cells;    /* cells of the liveness bitmap (gs_tile_quads), or 0: none (a memory budget) */
  int32_t flag_groups;   /* slot flags per entry: the backward's partial groups per batch */
} gs_frame_buffers;
size_t gs_frame_workspace_bytes(int32_t n, int32_t width, int32_t height, int32_t tile_size);
size_t gs_tile_workspace_bytes(int64_t capacity, int32_t num_tiles, int32_t live_cells, int32_t flag_groups);

typedef struct gs_render_fwd_args {
  gs_camera cam;
  gs_gaussians g;
  float *means2d, *conics, *radii; /* outputs, as gs_project_args */
  uint8_t *vis;
  float *image, *alpha, *depth;    /* outputs, as gs_blend_fwd_args */
  gs_frame_buffers fb;
  uint32_t key_base;               /* the depth-key window (gs_project_args) */
  int32_t key_bits;
  int32_t depth_sort_msd;          /* 1: gs_depth_sort_msd for windows of 9..31 bits */
  int32_t zero_slot_flags;         /* a backward follows: clear its slot flags [T, flag_groups] */
  uint32_t *host_counters_dev;     /* pinned [8] u32: device address (gs_bin_args.host_counters) */
  volatile uint32_t *host_counters_host; /* ... and host address of the same buffer */
  uint32_t host_seq;               /* this frame's sequence word (never the previous frame's) */
  uint32_t *pair_counts;           /* optional, gs_blend_fwd_args.pair_counts */
  uint32_t *pix_neval;             /* optional, gs_blend_fwd_args.pix_neval */
  int32_t resume;                  /* 1: continue after GS_NEED_CAPACITY, with a tile workspace of >= T */
  int32_t poll_timeout_ms;         /* the counter poll's patience before it synchronises the stream and
                                      looks once more (0: 10 s) */
  /* Device-resident frame (device_counts = 1): no host read-back at all.  The
   * count's status (GS_FRAME_*) and T stay on the device: the tile sort, the
   * ranges and the blend are launched for `capacity` entries (needs a tile
   * workspace) and read T themselves; a failed frame is drawn with empty
   * lists and flagged in counters[4] (and *step_flags).  The call returns
   * GS_OK with M, T unknown; the host reads (M, T, depth range, seq, status)
   * from the pinned counters whenever it likes.  For graph capture. */
  int32_t device_counts;
  uint32_t *step_flags;            /* optional, gs_bin_args.step_flags */
  uint32_t *frame_seq;             /* optional, gs_bin_args.frame_seq */
  /* results (and state for resume / the backward) */
  int32_t M, T;
  uint32_t depth_min_bits, depth_max_bits; /* counters[2..3] */
  int32_t depth_alt, tile_alt;
} gs_render_fwd_args;
/* GS_OK; M == 0: nothing drawn (renderer.py:74-83's background image is the
 * caller's); GS_NEED_CAPACITY / GS_RETRY_FULL_KEYS: see gs_status. */
gs_status gs_render_forward(gs_render_fwd_args *a, gs_stream_t stream);

typedef struct gs_render_bwd_args {
  gs_camera cam;
  gs_gaussians g;
  gs_frame_buffers fb;             /* the forward's */
  int32_t M, T, tile_alt;          /* the forward's results */
  const float *means2d, *conics;   /* the forward's outputs */
  const uint8_t *vis;
  const float *image, *alpha, *depth; /* the forward's outputs, unmodified (the blend backward reads them) */
  const float *g_image, *g_alpha, *g_depth; /* pixel cotangents (g_image NULL: none) */
  const float *g_means2d, *g_conics;        /* optional */
  float *pair_grads;               /* [T * fb.flag_groups, GS_PARTIAL_STRIDE] scratch */
  int32_t flags_zeroed;            /* the forward cleared the slot flags (zero_slot_flags) */
  int32_t project;                 /* 1: also run gs_project_backward over every Gaussian */
  float *d_xyz, *d_cov3d, *d_scaling, *d_rotation, *d_color_logits, *d_opacity, *d_sh_rest; /* as gs_project_bwd_args */
  float *grad_sums;                /* result: [n, 10] gathered sums in the frame workspace (for a
                                      caller's own gs_project_backward, e.g. per row range) */
  void *blend_events[2];           /* optional hipEvent_t pair, recorded on the stream right before and
                                      after the blend backward launch(es): its time alone (profiling) */
  int32_t device_counts;           /* the forward was device-resident: M, T are not read; pair_grads holds
                                      capacity * flag_groups partials (a failed frame gathers zero slots) */
  const gs_adam_args *fused_adam;  /* with project = 1: gs_project_backward_adam with these tensors (no
                                      d_* written), or NULL: the plain projection backward */
} gs_render_bwd_args;
gs_status gs_render_backward(gs_render_bwd_args *a, gs_stream_t stream);
/* Byte offsets of the buffers inside the two workspaces (for diagnostics and
 * tests that inspect a frame): frame -- records, rects, depth keys [2,n],
 * depth ids [2,n], key_minmax, counters, sort workspace, binning workspace,
 * pair_offset, tile ranges, pixel clamp flags, per-cell evaluated entries
 * (gs_blend_fwd_args.pix_flags / cell_neval), grad_sums, total; tile -- tile
 * keys (two halves), Gaussian ids (two halves), sort workspace, liveness
 * bitmap, slot flags, total, liveness words per cell. */
void gs_frame_offsets(int32_t n, int32_t width, int32_t height, int32_t tile_size, size_t out[14]);
void gs_tile_offsets(int64_t capacity, int32_t num_tiles, int32_t live_cells, int32_t flag_groups, size_t out[9]);

/* ---- misc --------------------------------------------------------------- */
int32_t gs_abi_version(void);
const char *gs_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* GSPLAT_MI355X_H */
