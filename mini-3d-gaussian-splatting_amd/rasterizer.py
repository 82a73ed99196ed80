"""Device pipeline + autograd for the render path.

One `render` = the reference's four stages (renderer.py:31-114):
  gs_project_forward   _project_gaussians_3d_to_2d + _frustum_culling
  gs_radix_sort_pairs  _sort_gaussians_by_depth (32-bit depth keys)
  gs_bin_count/emit    tile binning in depth order  (_tile_rasterization :263-298)
  gs_radix_sort_pairs  stable sort of the entries by tile id
  gs_tile_ranges       per-tile lists
  gs_blend_forward     per-pixel compositing        (:273-367)
and the backward: gs_blend_backward + gs_project_backward.

All buffers are torch tensors from the caching allocator; the HIP library
never allocates.  One host synchronisation per forward reads the visible
count M and the tile-touch count T (needed to size the entry buffers, and
for the reference's `vis_mask.sum() == 0` early return, renderer.py:74-83).
"""
from __future__ import annotations

import ctypes as C
import math
import os
import threading
import time
from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from . import _native as N


@dataclass
class CameraParams:
    """Host-side scalars of one view, as renderer.py:140-152 derives them."""
    image_width: int
    image_height: int
    fx: float
    fy: float
    cx: float
    cy: float
    view: Tuple[float, ...]  # 12 floats, rows 0..2 of the W2C matrix
    bg: Tuple[float, float, float]
    radius_min: float = 0.01
    radius_max: float = 50.0
    tile_size: int = N.GS_DEFAULT_TILE  # GaussianRenderer(tile_size) (renderer.py:24,261-264)

    @property
    def tiles_x(self) -> int:
        return (self.image_width + self.tile_size - 1) // self.tile_size

    @property
    def tiles_y(self) -> int:
        return (self.image_height + self.tile_size - 1) // self.tile_size

    @property
    def cells(self) -> int:
        """8x8 pixel cells per tile (gs_tile_quads): 4 at the default 16."""
        q = (self.tile_size + N.GS_QUAD - 1) // N.GS_QUAD
        return q * q

    @property
    def groups(self) -> int:
        """Gradient partials a one-batch blend backward writes per list entry
        (gs_partial_groups): one per 8x8 cell, 4 at the default tile.  Tiles
        of many cells may replay them in batches (frame_groups)."""
        return _partial_groups(self.tile_size)

    def frame_groups(self, entries: int) -> int:
        """Partials per entry of one backward batch for a frame of `entries`
        list entries: the combined default tile's one, else cell_batch."""
        return self.groups if self.groups < self.cells else cell_batch(self.cells, entries)

    def to_struct(self) -> N.GsCamera:
        """The ABI camera (cached per distinct value set: building it costs
        ~5-10 us of host time per frame; callers copy it into their
        argument structs and never modify it)."""
        key = (self.image_width, self.image_height, self.fx, self.fy, self.cx, self.cy, self.view, self.bg,
               self.radius_min, self.radius_max, self.tile_size)
        c = _CAM_STRUCTS.get(key)
        if c is None:
            if len(_CAM_STRUCTS) >= 4096:
                _CAM_STRUCTS.clear()
            c = _CAM_STRUCTS[key] = self._build_struct()
        return c

    def _build_struct(self) -> N.GsCamera:
        c = N.GsCamera()
        c.image_width, c.image_height = int(self.image_width), int(self.image_height)
        c.fx, c.fy, c.cx, c.cy = self.fx, self.fy, self.cx, self.cy
        c.view = (C.c_float * 12)(*self.view)
        c.radius_min, c.radius_max = self.radius_min, self.radius_max
        c.bg = (C.c_float * 3)(*self.bg)
        c.tile_size = int(self.tile_size)
        c.campos = (C.c_float * 3)(*self.campos)
        return c

    @property
    def campos(self) -> Tuple[float, float, float]:
        """Camera centre in world coordinates, -R^T t of the W2C view (the SH
        view direction's origin)."""
        v = self.view
        R = ((v[0], v[1], v[2]), (v[4], v[5], v[6]), (v[8], v[9], v[10]))
        t = (v[3], v[7], v[11])
        return tuple(-(R[0][j] * t[0] + R[1][j] * t[1] + R[2][j] * t[2]) for j in range(3))


_GROUPS: dict = {}
_CAM_STRUCTS: dict = {}  # CameraParams values -> GsCamera (CameraParams.to_struct)


def _partial_groups(tile_size: int) -> int:
    g = _GROUPS.get(tile_size)
    if g is None:
        g = _GROUPS[tile_size] = int(N.load().gs_partial_groups(int(tile_size)))
    return g


# Memory budgets for tiles of many 8x8 cells (the default tile's four cells
# never batch, the performance path): the backward's [T, G] partials + flags
# per cell batch, and the forward's [cells, live_words] liveness bitmap
# (above it none is written and the backward replays every entry).
PARTIAL_BUDGET_BYTES = int(os.environ.get("GS_PARTIAL_BUDGET", str(2 << 30)))
LIVE_BUDGET_BYTES = int(os.environ.get("GS_LIVE_BUDGET", str(1 << 30)))
_ALWAYS_ONE_BATCH = 4  # cells


def cell_batch(cells: int, entries: int) -> int:
    """Cells per blend-backward batch for a frame of `entries` list entries:
    every cell at once unless the [entries, cells] partials (40 B) and flags
    (1 B) would exceed PARTIAL_BUDGET_BYTES; batches are summed in order by
    gs_gather_partials (deterministic, bounded memory)."""
    per = 41 * max(int(entries), 1)
    if cells <= _ALWAYS_ONE_BATCH or cells * per <= PARTIAL_BUDGET_BYTES:
        return cells
    return max(1, min(cells, PARTIAL_BUDGET_BYTES // per))


def flag_bytes(cells: int, cap: int, groups: int = 0) -> int:
    """Slot-flag bytes that hold [T, frame_groups(T)] for every T <= cap (the
    batch is chosen from the frame's own T, so that the summation order, and
    with it every gradient bit, depends on the frame only -- not on the
    capacity guess of the frame before).  groups: gs_partial_groups."""
    if 0 < groups < cells:
        return groups * cap  # (combined cells: one batch)
    if cells <= _ALWAYS_ONE_BATCH:
        return cells * cap
    return max(min(cells * cap, PARTIAL_BUDGET_BYTES // 41), cap)


def live_bitmap_bytes(lib, cells: int, entries: int, num_tiles: int) -> int:
    """Bytes of the forward's liveness bitmap, or 0 when it exceeds
    LIVE_BUDGET_BYTES (then none is written; ADVICE r04: at 1080p a tile of
    1920 px holds 57,600 cells, ~7 GB of bitmap for 1M Gaussians)."""
    nbytes = 8 * cells * int(lib.gs_blend_live_words(int(entries), int(num_tiles)))
    return nbytes if cells <= _ALWAYS_ONE_BATCH or nbytes <= LIVE_BUDGET_BYTES else 0


def _rows(t: torch.Tensor, cols: int) -> Tuple[torch.Tensor, int]:
    """(tensor, row stride in floats) without copying when rows are dense."""
    if t.dim() == 1 and cols == 1:
        return t, t.stride(0)
    if t.stride(-1) != 1 or t.shape[-1] != cols:
        t = t.contiguous()
    return t, t.stride(0)


_G_STRUCTS: dict = {}  # (pointers, strides, flags) -> GsGaussians (_gaussians_struct)


def _gaussians_struct(n, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit=False,
                      sh_rest=None, sh_degree=0) -> N.GsGaussians:
    """The ABI view of the Gaussians' tensors, cached by the addresses,
    strides and flags it holds (the same model renders with the same struct;
    callers copy it and never modify it)."""
    key = (n, xyz.data_ptr(), xyz.stride(0), None if cov3d is None else cov3d.data_ptr(),
           None if scaling is None else scaling.data_ptr(), None if rotation is None else rotation.data_ptr(),
           logits.data_ptr(), logits.stride(0), opacity.data_ptr(), opacity.stride(0), bool(opacity_is_logit),
           int(sh_degree), None if sh_rest is None or sh_degree <= 0 else (sh_rest.data_ptr(), sh_rest.stride(0)))
    g = _G_STRUCTS.get(key)
    if g is None:
        if len(_G_STRUCTS) >= 4096:
            _G_STRUCTS.clear()
        g = _G_STRUCTS[key] = _build_gaussians_struct(n, xyz, cov3d, scaling, rotation, logits, opacity,
                                                      opacity_is_logit, sh_rest, sh_degree)
    return g


def _build_gaussians_struct(n, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit=False,
                            sh_rest=None, sh_degree=0) -> N.GsGaussians:
    g = N.GsGaussians()
    g.n = n
    g.xyz, g.xyz_stride = N.ptr(xyz), xyz.stride(0)
    g.cov3d = N.ptr(cov3d)
    g.scaling, g.rotation = N.ptr(scaling), N.ptr(rotation)
    g.color_logits, g.color_stride = N.ptr(logits), logits.stride(0)
    g.opacity, g.opacity_stride = N.ptr(opacity), opacity.stride(0)
    g.opacity_is_logit = 1 if opacity_is_logit else 0
    if sh_degree > 0:
        g.sh_degree, g.sh_rest, g.sh_rest_stride = int(sh_degree), N.ptr(sh_rest), sh_rest.stride(0)
    return g


def _stream() -> int:
    return N.stream_ptr()


class StageTimer:
    """Optional per-stage HIP-event timing on the stream the kernels are
    launched on (torch's current stream).  Disabled unless a bench enables it;
    when disabled, mark() is a no-op."""
    enabled = False
    only = None  # optional set of stage names to record (the others cost nothing)
    events: list = []
    pairs: list = []  # (name, e0, e1): intervals the library records around one launch (pair())
    _pool: list = []  # created events, reused across resets (creating one costs more host time than recording)
    _used = 0
    _raw: list = []   # N.RawEvent pool for pair()
    _raw_used = 0

    @classmethod
    def _event(cls):
        if cls._used == len(cls._pool):
            cls._pool.append(torch.cuda.Event(enable_timing=True))
        e = cls._pool[cls._used]
        cls._used += 1
        return e

    @classmethod
    def mark(cls, name: str):
        if cls.enabled and (cls.only is None or name in cls.only):
            e = cls._event()
            e.record()
            cls.events.append((name, e))

    @classmethod
    def pair(cls, name: str):
        """(e0, e1) for a launch the library brackets itself (the frame
        backward's blend launch), or None when `name` is not timed."""
        if not (cls.enabled and (cls.only is None or name in cls.only)):
            return None
        while len(cls._raw) < cls._raw_used + 2:
            cls._raw.append(N.RawEvent())
        e0, e1 = cls._raw[cls._raw_used], cls._raw[cls._raw_used + 1]
        cls._raw_used += 2
        cls.pairs.append((name, e0, e1))
        return e0, e1

    @classmethod
    def reset(cls):
        cls.events, cls.pairs, cls._used, cls._raw_used = [], [], 0, 0

    @classmethod
    def durations_ms(cls):
        """{stage: [ms per occurrence]} -- stage = interval from its mark to
        the next, or a bracketed launch's own interval."""
        torch.cuda.synchronize()
        out = {}
        ev = cls.events
        for (name, e0), (_, e1) in zip(ev[:-1], ev[1:]):
            if name.startswith("~"):
                continue
            out.setdefault(name, []).append(e0.elapsed_time(e1))
        for name, e0, e1 in cls.pairs:
            out.setdefault(name, []).append(e0.elapsed_ms(e1))
        return out


def _check_inputs(xyz: torch.Tensor):
    if not xyz.is_cuda:
        raise RuntimeError("the MI355X renderer needs Gaussians on a HIP device (got %s); "
                           "there is no CPU path" % xyz.device)


class _Frame:
    """Intermediate device buffers of one forward, kept for the backward."""
    __slots__ = ("records", "rects", "vis", "pair_offset", "order", "ranges", "sorted_gauss", "pix_flags",
                 "cell_neval", "live_bits", "big", "M", "T", "slot_live", "groups", "consumed")


_T_SEEN: dict = {}  # device -> tile entries T of its last frame (capacity guess)
# per host thread: device -> pinned int32[4] for the (M, T, depth-bits range)
# read-back (renders from several threads each read their own counters; the
# two per-device guesses above are only guesses, a stale one is corrected)
_HOST_COUNTERS = threading.local()


class _HostCounters:
    """Pinned int32[8] gs_bin_count writes (M, T, depth-bits min / max) and
    then a sequence word into, through its device address: the host polls the
    word -- no copy and no event in the stream (an event record between the
    count and the emission cost a ~6 us gap on the GPU).  Without a device
    address (dptr None) the counters are copied and an event is waited for."""
    __slots__ = ("t", "np", "dptr", "seq")

    def __init__(self):
        self.t = torch.empty((8,), dtype=torch.int32, pin_memory=True)
        self.np = self.t.numpy()
        self.dptr = N.host_device_pointer(self.t)
        self.seq = 0

    def arm(self, ba) -> None:
        if self.dptr is None:
            return
        self.seq = self.seq % 0x7FFFFFFF + 1
        self.np[4] = 0  # (the previous frame's word; the GPU writes this frame's after its counters)
        ba.host_counters, ba.host_seq = self.dptr, self.seq

    def wait(self, dev, ready) -> Tuple[int, int, int, int]:
        if self.dptr is None:
            ready.synchronize()
        else:
            hv, seq, i = self.np, self.seq, 0
            deadline = time.perf_counter() + 10.0
            while hv[4] != seq:
                i += 1
                if (i & 255) == 0:
                    if time.perf_counter() > deadline:  # (never in a healthy run)
                        torch.cuda.synchronize(dev)
                        if hv[4] != seq:
                            raise RuntimeError("gs_bin_count: the frame's counters never reached the host")
                        break
                    time.sleep(0)  # other host threads get the interpreter
        v = self.np[:4].tolist()
        return int(v[0]), int(v[1]), int(v[2]) & 0xFFFFFFFF, int(v[3]) & 0xFFFFFFFF
_FUSE_FLAGS = os.environ.get("GS_FUSE_SLOT_FLAGS", "1") != "0"  # slot flags zeroed by gs_tile_ranges
# Depth-key windows (per process and device; these are guesses, a stale one
# only costs a re-render, so host threads may race on them): the window
# covers the union of the last _WINDOW_FRAMES frames' visible depth ranges, so
# views that alternate (a trainer's shuffled cameras) keep fitting it.  A
# frame whose depths leave the window (a miss) is rendered again with 32-bit
# keys; a second miss within _MISS_SPAN frames turns windows off for
# _WINDOW_OFF_FRAMES frames (a miss costs a whole re-render, a window saves
# ~20 us of sorting).
_DEPTH_HIST: dict = {}  # device -> [(zmin_bits, zmax_bits)] of its last frames
_WINDOW_FRAMES = 8
_MISS_SPAN = 32
_WINDOW_OFF_FRAMES = 256
_WINDOW_STATE: dict = {}  # device -> {"frame", "misses", "last_miss", "off_until"}
# Windowed depth keys of 9..31 bits are sorted by gs_depth_sort_msd (one MSD pass + a sort per
# bucket in LDS) unless GS_DEPTH_MSD=0.  A bucket over its LDS capacity (clumped depths) poisons
# the frame's depth max (0xFFFFFFFF): the frame is sorted again with the LSD passes, and the LSD
# path is kept for the next _MSD_BACKOFF_FRAMES frames on that device.
_DEPTH_MSD = os.environ.get("GS_DEPTH_MSD", "1") != "0"
_MSD_BACKOFF: dict = {}  # device -> frames left on the LSD path after an overflow
_MSD_BACKOFF_FRAMES = 64
_POISON = 0xFFFFFFFF


def depth_window(zmin_bits: int, zmax_bits: int):
    """(key_base, key_bits) of a window around the visible fp32 depth bits
    [zmin_bits, zmax_bits], widened by 1/8 of the range on both sides for the
    next frame's drift; None when the range needs all 32 bits.  Windows of 25-31
    bits save no LSD pass, but they keep the depth sort on gs_depth_sort_msd
    (raw fp32 bits would put every key into one MSD bucket)."""
    if zmin_bits > zmax_bits:
        return None
    span = zmax_bits - zmin_bits
    lo = max(0, zmin_bits - span // 8 - 1)
    hi = zmax_bits + span // 8 + 1
    bits = max(1, (hi - lo + 1).bit_length())  # keys 0 .. hi - lo < 2^bits - 1 (the culled sentinel)
    if bits >= 9 and hi - lo >= _msd_limit(bits):
        bits += 1  # the MSD depth sort's top bucket is the sentinel's alone
    return (lo, bits) if bits < 32 else None


def _msd_limit(bits: int) -> int:
    """Visible keys of a `bits`-bit window stay below this: 2^bits - 1 (the
    culled sentinel) and, from 9 bits on, 255 << (bits - 8), so that the top
    digit of gs_depth_sort_msd's MSD pass holds the sentinel only."""
    return min((1 << bits) - 1, 255 << (bits - 8)) if bits >= 9 else (1 << bits) - 1


def _window_state(dev) -> dict:
    st = _WINDOW_STATE.get(dev)
    if st is None:
        st = _WINDOW_STATE[dev] = {"frame": 0, "misses": 0, "last_miss": None, "off_until": 0}
    return st


def _window_for(dev):
    """The depth-key window of this device's next frame (None: 32-bit keys)."""
    st = _window_state(dev)
    hist = _DEPTH_HIST.get(dev)
    if not hist or st["frame"] < st["off_until"]:
        return None
    return depth_window(min(h[0] for h in hist), max(h[1] for h in hist))


def _record_depths(dev, zmin_bits: int, zmax_bits: int) -> None:
    """A finished frame's visible depth-bit range (none visible: nothing)."""
    st = _window_state(dev)
    st["frame"] += 1
    if zmin_bits > zmax_bits:
        return
    hist = _DEPTH_HIST.setdefault(dev, [])
    hist.append((zmin_bits, zmax_bits))
    del hist[:-_WINDOW_FRAMES]


def _note_window_miss(dev) -> None:
    st = _window_state(dev)
    st["misses"] += 1
    if st["last_miss"] is not None and st["frame"] - st["last_miss"] <= _MISS_SPAN:
        st["off_until"] = st["frame"] + _WINDOW_OFF_FRAMES
    st["last_miss"] = st["frame"]


def depth_window_stats(dev=None) -> dict:
    """Frames rendered and window misses (re-renders) per device: a
    measurement of the depth-key window's hit rate."""
    if dev is not None:
        return dict(_window_state(torch.device(dev)))
    return {str(d): dict(v) for d, v in _WINDOW_STATE.items()}


def window_holds(window, zmin_bits: int, zmax_bits: int) -> bool:
    """Did every visible key of this frame fit the window it was sorted with?"""
    if window is None or zmin_bits > zmax_bits:
        return True
    base, bits = window
    return zmin_bits >= base and zmax_bits - base < _msd_limit(bits)


def _alloc_tile_buffers(lib, cap: int, num_tiles: int, cam: CameraParams, dev):
    """One byte buffer for T <= cap entries: tile keys + Gaussian ids
    (ping-pong, 16 B/entry), the tile sort's workspace, the liveness bitmap
    (cells x gs_blend_live_words, within LIVE_BUDGET_BYTES) and the backward's
    slot flags (the first cell batch's groups, B/entry)."""
    nbytes = (16 * cap + 255) // 256 * 256
    nbytes += (int(lib.gs_radix_sort_workspace_bytes(cap)) + 255) // 256 * 256
    nbytes += live_bitmap_bytes(lib, cam.cells, cap, num_tiles)
    nbytes += (flag_bytes(cam.cells, cap, cam.groups) + 255) // 256 * 256  # slot flags (zeroed by gs_tile_ranges)
    return torch.empty((nbytes,), dtype=torch.uint8, device=dev), cap


class _TileLayout:
    """Addresses inside one _alloc_tile_buffers allocation of capacity `cap`:
    tile keys and Gaussian ids (ping-pong), the tile sort's workspace, the
    liveness bitmap (stride live_words, sized for `cap` entries)."""
    __slots__ = ("big", "cap", "p_tk", "p_tv", "p_ws", "ws_bytes", "o_live", "p_live", "live_words", "bits",
                 "o_flags", "groups")


def _tile_layout(lib, buf, num_tiles: int, cam: CameraParams) -> _TileLayout:
    big, cap = buf
    L = _TileLayout()
    L.big, L.cap = big, cap
    base = big.data_ptr()
    L.p_tk = (base, base + 4 * cap)             # tile keys, ping-pong
    L.p_tv = (base + 8 * cap, base + 12 * cap)  # Gaussian ids, ping-pong
    o_ws = (16 * cap + 255) // 256 * 256
    L.ws_bytes = int(lib.gs_radix_sort_workspace_bytes(cap))  # (>= what any T <= cap needs)
    L.o_live = o_ws + (L.ws_bytes + 255) // 256 * 256
    live_bytes = live_bitmap_bytes(lib, cam.cells, cap, num_tiles)
    L.p_ws, L.p_live = base + o_ws, (base + L.o_live if live_bytes else None)
    L.live_words = int(lib.gs_blend_live_words(cap, num_tiles)) if live_bytes else 0
    L.o_flags = L.o_live + live_bytes
    L.groups = 0  # the backward's partials per entry and batch: frame_groups(T), set once T is known
    L.bits = max(1, int(math.ceil(math.log2(num_tiles))) if num_tiles > 1 else 1)
    return L


# Frames at the default tile run through the library's frame entry points
# (gs_render_forward / gs_render_backward: one call per direction over two
# workspaces, ABI 18) unless GS_FRAME_CALLS=0; other tile sizes, and hosts
# whose pinned counters have no device address, take the stage-by-stage path
# below.  The two paths launch the same kernels on the same data: their
# outputs and gradients are bit-identical (test_frame_entry_points_match).
_FRAME_CALLS = os.environ.get("GS_FRAME_CALLS", "1") != "0"
# gs_render_forward's patience with the counter poll before it synchronises the
# stream and looks once more (0: the library's 10 s; tests shorten it)
_POLL_TIMEOUT_MS = int(os.environ.get("GS_POLL_TIMEOUT_MS", "0"))
_WS_BYTES: dict = {}  # (n, W, H, tile) -> gs_frame_workspace_bytes


class _FastFrame:
    """One forward's state for its backward, in the frame and tile
    workspaces (gs_render_forward).  The buffers the tests and the bench
    inspect are views made on demand (gs_frame_offsets / gs_tile_offsets)."""
    __slots__ = ("fa", "frame_ws", "tile_ws", "M", "T", "groups", "_off", "_toff", "n", "HW", "tiles", "cells",
                 "slot_live_zeroed", "vis")

    def _o(self):
        if self._off is None:
            lib = N.load()
            fo = (C.c_size_t * 14)()
            c = self.fa.cam
            lib.gs_frame_offsets(self.n, c.image_width, c.image_height, c.tile_size, fo)
            to = (C.c_size_t * 9)()
            fb = self.fa.fb
            lib.gs_tile_offsets(fb.capacity, self.tiles, fb.live_cells, fb.flag_groups, to)
            self._off, self._toff = list(fo), list(to)
        return self._off, self._toff

    def _f(self, i, nbytes, dtype, shape):
        o = self._o()[0][i]
        return self.frame_ws[o:o + nbytes].view(dtype).view(shape)

    def _t(self, i, nbytes, dtype, shape):
        o = self._o()[1][i]
        return self.tile_ws[o:o + nbytes].view(dtype).view(shape)

    records = property(lambda s: s._f(0, 4 * N.GS_RECORD_FLOATS * s.n, torch.float32, (s.n, N.GS_RECORD_FLOATS)))
    rects = property(lambda s: s._f(1, 8 * s.n, torch.int32, (s.n, 2)))
    order = property(lambda s: s._f(3, 8 * s.n, torch.int32, (2, s.n))[s.fa.depth_alt])
    pair_offset = property(lambda s: s._f(8, 4 * s.n, torch.int32, (s.n,)))
    ranges = property(lambda s: s._f(9, 8 * s.tiles, torch.int32, (s.tiles, 2)))
    pix_flags = property(lambda s: s._f(10, s.HW, torch.uint8, (s.HW,)))
    cell_neval = property(lambda s: s._f(11, 4 * s.tiles * s.cells, torch.int32, (s.tiles, s.cells)))
    sorted_gauss = property(lambda s: s._t(2 + s.fa.tile_alt, 4 * s.T, torch.int32, (s.T,)))
    live_bits = property(lambda s: s._t(5, 8 * s.cells * s._o()[1][8], torch.int64, (s.cells, s._o()[1][8])))
    slot_live = property(lambda s: s._t(6, s.groups * s.T, torch.uint8, (s.groups * s.T,)))



def _host_counters(dev) -> "_HostCounters":
    per_thread = getattr(_HOST_COUNTERS, "bufs", None)
    if per_thread is None:
        per_thread = _HOST_COUNTERS.bufs = {}
    hc = per_thread.get(dev)
    if hc is None:
        hc = per_thread[dev] = _HostCounters()
    return hc


def _forward_frame(cam: CameraParams, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit, sh_rest,
                   sh_degree, pair_counts, depth_window_ok, need_grad, hc, pix_neval):
    """forward_pipeline through gs_render_forward (the default tile)."""
    lib = N.load()
    dev = xyz.device
    n = int(xyz.shape[0])
    H, W = int(cam.image_height), int(cam.image_width)
    f32 = torch.float32
    s = _stream()
    tiles = cam.tiles_x * cam.tiles_y
    key = (n, W, H, cam.tile_size)
    fws = _WS_BYTES.get(key)
    if fws is None:
        fws = _WS_BYTES[key] = int(lib.gs_frame_workspace_bytes(n, W, H, cam.tile_size))
    fa = N.GsRenderFwdArgs()
    fa.cam = cam.to_struct()
    fa.g = _gaussians_struct(n, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit, sh_rest, sh_degree)
    means2d = torch.empty((n, 2), dtype=f32, device=dev)
    conics = torch.empty((n, 2, 2), dtype=f32, device=dev)
    radii = torch.empty((n,), dtype=f32, device=dev)
    vis = torch.empty((n,), dtype=torch.bool, device=dev)
    image = torch.empty((3, H, W), dtype=f32, device=dev)
    alpha = torch.empty((1, H, W), dtype=f32, device=dev)
    depth = torch.empty((1, H, W), dtype=f32, device=dev)
    frame_ws = torch.empty((fws,), dtype=torch.uint8, device=dev)
    fa.means2d, fa.conics, fa.radii, fa.vis = (means2d.data_ptr(), conics.data_ptr(), radii.data_ptr(),
                                               vis.data_ptr())
    fa.image, fa.alpha, fa.depth = image.data_ptr(), alpha.data_ptr(), depth.data_ptr()
    fb = fa.fb
    fb.frame_ws, fb.frame_ws_bytes = frame_ws.data_ptr(), fws
    fb.live_cells, fb.flag_groups = cam.cells, cam.groups
    cap = _T_SEEN.get(dev, 0)
    cap = cap + cap // 4 + 4096 if cap else 0
    tile_ws = None
    if cap:
        tws = int(lib.gs_tile_workspace_bytes(cap, tiles, cam.cells, cam.groups))
        tile_ws = torch.empty((tws,), dtype=torch.uint8, device=dev)
        fb.tile_ws, fb.tile_ws_bytes, fb.capacity = tile_ws.data_ptr(), tws, cap
    window = _window_for(dev) if depth_window_ok else None
    fa.key_base, fa.key_bits = window if window is not None else (0, 32)
    msd = _DEPTH_MSD and window is not None and 9 <= fa.key_bits <= 31
    backoff = _MSD_BACKOFF.get(dev, 0)
    if msd and backoff:
        _MSD_BACKOFF[dev] = backoff - 1
    fa.depth_sort_msd = 1 if (msd and not backoff) else 0
    fa.zero_slot_flags = 1 if need_grad else 0
    hc.seq = hc.seq % 0x7FFFFFFF + 1
    fa.host_counters_dev, fa.host_counters_host, fa.host_seq = hc.dptr, hc.t.data_ptr(), hc.seq
    fa.pair_counts, fa.pix_neval = N.ptr(pair_counts), N.ptr(pix_neval)
    fa.poll_timeout_ms = _POLL_TIMEOUT_MS
    st = lib.gs_render_forward(C.byref(fa), s)
    if st == N.GS_RETRY_FULL_KEYS:
        # a visible depth outside the window, or an MSD bucket over capacity
        if fa.depth_max_bits == _POISON:
            _MSD_BACKOFF[dev] = _MSD_BACKOFF_FRAMES
        else:
            _note_window_miss(dev)
        _T_SEEN[dev] = fa.T
        return forward_pipeline(cam, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit,
                                sh_rest, sh_degree, pair_counts, depth_window_ok=False, need_grad=need_grad,
                                pix_neval=pix_neval)
    if st == N.GS_NEED_CAPACITY:
        cap = fa.T
        tws = int(lib.gs_tile_workspace_bytes(cap, tiles, cam.cells, cam.groups))
        tile_ws = torch.empty((tws,), dtype=torch.uint8, device=dev)
        fb.tile_ws, fb.tile_ws_bytes, fb.capacity = tile_ws.data_ptr(), tws, cap
        fa.resume = 1
        st = lib.gs_render_forward(C.byref(fa), s)
    N.check(st, "gs_render_forward")
    M, T = int(fa.M), int(fa.T)
    if n > 0:
        _T_SEEN[dev] = T
        _record_depths(dev, int(fa.depth_min_bits), int(fa.depth_max_bits))
    fr = _FastFrame()
    fr.fa, fr.frame_ws, fr.tile_ws, fr.M, fr.T = fa, frame_ws, tile_ws, M, T
    fr.groups, fr._off, fr._toff, fr.n, fr.HW, fr.tiles, fr.cells = cam.groups, None, None, n, H * W, tiles, cam.cells
    fr.slot_live_zeroed = bool(need_grad)
    fr.vis = vis
    if M == 0:
        # renderer.py:74-83: bg once (not doubled, not clamped), zero alpha/depth
        image = torch.tensor(cam.bg, dtype=f32, device=dev).view(3, 1, 1).repeat(1, H, W)
        alpha = torch.zeros((1, H, W), dtype=f32, device=dev)
        depth = torch.zeros((1, H, W), dtype=f32, device=dev)
    return image, alpha, depth, means2d, conics, radii, vis, fr


def forward_pipeline(cam: CameraParams, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit=False,
                     sh_rest=None, sh_degree=0, pair_counts=None, depth_window_ok=True, need_grad=False,
                     pix_neval=None):
    """pair_counts / pix_neval: optional int32 [H*W] the blend fills with each
    pixel's contributing pairs / evaluated entries (measurement counters,
    SURVEY 8d, and the oracle's decision-forced replay; not in render()).

    The depth sort runs over a window of the depth keys' bits chosen from the
    previous frame's visible depth range on this device (one radix pass less
    per 8 bits, gs_project_args.key_base); this frame's range, read back with
    (M, T), says whether the window held -- if not, the frame is rendered
    again with full 32-bit keys (depth_window_ok=False)."""
    if _FRAME_CALLS and cam.tile_size == N.GS_DEFAULT_TILE:
        hc = _host_counters(xyz.device)
        if hc.dptr is not None:
            return _forward_frame(cam, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit, sh_rest,
                                  sh_degree, pair_counts, depth_window_ok, need_grad, hc, pix_neval)
    lib = N.load()
    dev = xyz.device
    n = int(xyz.shape[0])
    H, W = int(cam.image_height), int(cam.image_width)
    f32, i32 = torch.float32, torch.int32
    s = _stream()
    cs = cam.to_struct()
    gst = _gaussians_struct(n, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit, sh_rest, sh_degree)

    means2d = torch.empty((n, 2), dtype=f32, device=dev)
    conics = torch.empty((n, 2, 2), dtype=f32, device=dev)
    radii = torch.empty((n,), dtype=f32, device=dev)
    vis = torch.empty((n,), dtype=torch.bool, device=dev)
    records = torch.empty((n, N.GS_RECORD_FLOATS), dtype=f32, device=dev)
    rects = torch.empty((n, 2), dtype=i32, device=dev)
    keys = torch.empty((2, n), dtype=i32, device=dev)
    vals = torch.empty((2, n), dtype=i32, device=dev)
    counters = torch.empty((N.GS_NUM_COUNTERS,), dtype=i32, device=dev)
    key_minmax = torch.empty((2 * max(1, (n + 255) // 256),), dtype=i32, device=dev)
    window = _window_for(dev) if depth_window_ok else None
    key_base, key_bits = window if window is not None else (0, 32)

    StageTimer.mark("project_fwd")
    pa = N.GsProjectArgs(cs, gst, N.ptr(means2d), N.ptr(conics), N.ptr(radii), N.ptr(vis), N.ptr(records),
                         N.ptr(rects), N.ptr(keys[0]), key_base, key_bits, N.ptr(key_minmax))
    N.check(lib.gs_project_forward(C.byref(pa), s), "gs_project_forward")

    fr = _Frame()
    fr.slot_live = None
    fr.consumed = False  # (a backward ran: the slot flags hold its last batch's, not the forward's zeros)
    fr.groups = cam.groups
    fr.records, fr.rects, fr.vis, fr.order = records, rects, vis, None
    if n > 0:
        ws = torch.empty((lib.gs_radix_sort_workspace_bytes(n),), dtype=torch.uint8, device=dev)
        StageTimer.mark("depth_sort")
        alt = C.c_int32(0)
        # (the MSD backoff counts only frames that would have taken the MSD
        # sort; it is per process and device, not per host thread)
        msd = _DEPTH_MSD and window is not None and 9 <= key_bits <= 31
        backoff = _MSD_BACKOFF.get(dev, 0)
        if msd and backoff:
            _MSD_BACKOFF[dev] = backoff - 1
        if msd and not backoff:
            N.check(lib.gs_depth_sort_msd(N.ptr(keys[0]), N.ptr(vals[0]), N.ptr(keys[1]), N.ptr(vals[1]), n,
                                          key_bits, N.ptr(ws), ws.numel(), N.ptr(key_minmax) + 4, C.byref(alt),
                                          s), "depth sort (msd)")
        else:
            N.check(lib.gs_radix_sort_pairs(N.ptr(keys[0]), N.ptr(vals[0]), N.ptr(keys[1]), N.ptr(vals[1]), n, 0,
                                            key_bits, 1, N.ptr(ws), ws.numel(), C.byref(alt), s), "depth sort")
        sorted_ids = vals[alt.value]
        fr.order = sorted_ids
        bws = torch.empty((lib.gs_bin_workspace_bytes(n),), dtype=torch.uint8, device=dev)
        pair_offset = torch.empty((n,), dtype=i32, device=dev)
        ba = N.GsBinArgs(n, cam.tiles_x, cam.tiles_y, N.ptr(sorted_ids), N.ptr(rects), N.ptr(vis),
                         N.ptr(counters), N.ptr(key_minmax), N.ptr(bws), bws.numel(), 0, 0, N.ptr(pair_offset),
                         N.ptr(records), 0)
        per_thread = getattr(_HOST_COUNTERS, "bufs", None)
        if per_thread is None:
            per_thread = _HOST_COUNTERS.bufs = {}
        hc = per_thread.get(dev)
        if hc is None:
            hc = per_thread[dev] = _HostCounters()
        hc.arm(ba)
        StageTimer.mark("bin_count")
        N.check(lib.gs_bin_count(C.byref(ba), s), "gs_bin_count")
        # everything whose size does not depend on T is allocated before the
        # one host sync, so the GPU waits only for the read-back and launches
        num_tiles = cam.tiles_x * cam.tiles_y
        ranges = torch.empty((num_tiles, 2), dtype=i32, device=dev)
        image = torch.empty((3, H, W), dtype=f32, device=dev)
        alpha = torch.empty((1, H, W), dtype=f32, device=dev)
        depth = torch.empty((1, H, W), dtype=f32, device=dev)
        pix_flags = torch.empty((H * W,), dtype=torch.uint8, device=dev)
        cell_neval = torch.empty((num_tiles, cam.cells), dtype=i32, device=dev)
        # the T-sized buffers too, at a capacity guessed from the last frame on
        # this device, and the emission queued into them before the sync (it
        # drops entries past the capacity): its kernel time hides the
        # read-back's round trip.  T above the guess: re-allocate, re-emit.
        cap = _T_SEEN.get(dev, 0)
        big_guess = _alloc_tile_buffers(lib, cap + cap // 4 + 4096, num_tiles, cam, dev) if cap else None
        # (M, T) reach the host through pinned memory before the emission is
        # queued, so the host wakes while the GPU still emits: gs_bin_count
        # writes them there itself (_HostCounters) -- or, where the runtime
        # does not map the buffer, a copy in the stream and an event
        ready = None
        if hc.dptr is None:
            hc.t[:4].copy_(counters[:4], non_blocking=True)
            ready = torch.cuda.Event()
            ready.record()
        if big_guess is not None:
            gb, gcap = big_guess[0].data_ptr(), big_guess[1]
            ba.tile_keys, ba.pair_gauss, ba.capacity = gb, gb + 8 * gcap, gcap
            StageTimer.mark("bin_emit")
            N.check(lib.gs_bin_emit(C.byref(ba), s), "gs_bin_emit")
            # everything the launches after the sync need but T, laid out now
            # (the GPU is emitting): after the sync only T is filled in
            layout = _tile_layout(lib, big_guess, num_tiles, cam)
        StageTimer.mark("~sync")
        M, T, zmin, zmax = hc.wait(dev, ready)  # the one host sync
        if not window_holds(window, zmin, zmax):
            # a visible depth outside the window (the sort's keys were clipped),
            # or an MSD bucket over capacity (the depth max poisoned)
            if zmax == _POISON:
                _MSD_BACKOFF[dev] = _MSD_BACKOFF_FRAMES
            else:
                _note_window_miss(dev)
            _T_SEEN[dev] = T
            return forward_pipeline(cam, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit,
                                    sh_rest, sh_degree, pair_counts, depth_window_ok=False, need_grad=need_grad,
                                    pix_neval=pix_neval)
    else:
        M, T = 0, 0
    fr.M, fr.T = M, T

    if M == 0:
        if n > 0:
            _T_SEEN[dev] = T
            _record_depths(dev, zmin, zmax)
        # renderer.py:74-83: bg once (not doubled, not clamped), zero alpha/depth
        bg = torch.tensor(cam.bg, dtype=f32, device=dev).view(3, 1, 1)
        image = bg.repeat(1, H, W)
        alpha = torch.zeros((1, H, W), dtype=f32, device=dev)
        depth = torch.zeros((1, H, W), dtype=f32, device=dev)
        fr.pair_offset = torch.zeros((max(n, 1),), dtype=i32, device=dev)
        return image, alpha, depth, means2d, conics, radii, vis, fr

    # Between the host sync and the blend launch the GPU idles: this span
    # only fills T into the prepared launches (re-emitting first when T
    # exceeded the guess); views of the buffers are made after the blend is
    # queued.
    emitted = big_guess is not None and big_guess[1] >= T
    if not emitted:
        layout = _tile_layout(lib, _alloc_tile_buffers(lib, T, num_tiles, cam, dev), num_tiles, cam)
        ba.tile_keys, ba.pair_gauss, ba.capacity = layout.p_tk[0], layout.p_tv[0], layout.cap
        StageTimer.mark("bin_emit")
        N.check(lib.gs_bin_emit(C.byref(ba), s), "gs_bin_emit")
    L = layout
    L.groups = cam.frame_groups(T)  # (from T alone: the gradients' summation order)
    assert L.groups * T <= flag_bytes(cam.cells, L.cap, cam.groups)
    alt = C.c_int32(0)
    StageTimer.mark("tile_sort")
    N.check(lib.gs_radix_sort_pairs(L.p_tk[0], L.p_tv[0], L.p_tk[1], L.p_tv[1], T, 0, L.bits, 0,
                                    L.p_ws, L.ws_bytes, C.byref(alt), s), "tile sort")
    # (with gradients to come: the backward's slot flags zeroed in the same kernel)
    ra = N.GsRangeArgs(T, num_tiles, L.p_tk[alt.value], N.ptr(ranges),
                       L.big.data_ptr() + L.o_flags if need_grad else None, L.groups)
    StageTimer.mark("tile_ranges")
    N.check(lib.gs_tile_ranges(C.byref(ra), s), "gs_tile_ranges")

    fa = N.GsBlendFwdArgs(cs, cam.tiles_x, cam.tiles_y, N.ptr(ranges), L.p_tv[alt.value], N.ptr(records),
                          N.ptr(image), N.ptr(alpha), N.ptr(depth), N.ptr(pix_flags), N.ptr(cell_neval),
                          L.p_live, L.live_words, N.ptr(pair_counts), T, N.ptr(pix_neval))
    StageTimer.mark("blend_fwd")
    N.check(lib.gs_blend_forward(C.byref(fa), s), "gs_blend_forward")
    StageTimer.mark("~end_fwd")
    _T_SEEN[dev] = T  # (the next frame's guesses: after the launches)
    _record_depths(dev, zmin, zmax)

    # (the blend is queued: views for the frame cost no GPU idle time now)
    kv = L.big[:16 * L.cap].view(i32).view(4, L.cap)
    fr.sorted_gauss = kv[2 + alt.value, :T]
    fr.live_bits = (L.big[L.o_live:L.o_live + 8 * cam.cells * L.live_words].view(torch.int64)
                    .view(cam.cells, L.live_words) if L.live_words else None)
    fr.big = L.big
    fr.groups = L.groups
    fr.slot_live = L.big[L.o_flags:L.o_flags + L.groups * T] if need_grad else None
    fr.pair_offset, fr.ranges = pair_offset, ranges
    fr.pix_flags, fr.cell_neval = pix_flags, cell_neval
    return image, alpha, depth, means2d, conics, radii, vis, fr


def backward_pipeline(cam: CameraParams, fr: _Frame, xyz, cov3d, scaling, rotation, logits, opacity,
                      means2d, conics, g_image, g_alpha, g_depth, g_means2d, g_conics, opacity_is_logit=False,
                      sh_rest=None, sh_degree=0, out=None, outputs=None):
    """outputs: the forward's (image, alpha, depth), unmodified -- with the
    frame's clamp flags they are the blend backward's per-pixel state.
    out: optional preallocated gradient tensors {name: tensor} (the
    data-parallel bucket's views, distributed.GradAllReduce.attach); the
    kernels write there instead of into fresh buffers.  out["_rows_ready"]
    (optional): called with (lo, hi) once the gradient rows of Gaussians
    [lo, hi) are queued, the last stage running in out["_chunks"] ranges so
    that a range's all-reduce overlaps the next range's kernels."""
    if isinstance(fr, _FastFrame):
        return _backward_frame(cam, fr, xyz, cov3d, scaling, rotation, logits, opacity, means2d, conics, g_image,
                               g_alpha, g_depth, g_means2d, g_conics, opacity_is_logit, sh_rest, sh_degree, out,
                               outputs)
    lib = N.load()
    dev = xyz.device
    n = int(xyz.shape[0])
    f32 = torch.float32
    s = _stream()
    cs = cam.to_struct()
    pair_grads = slot_live = None
    pixel_grads = g_image is not None or g_alpha is not None or g_depth is not None
    if fr.M > 0 and fr.T > 0 and pixel_grads:
        if g_image is None:
            g_image = torch.zeros((3, cam.image_height, cam.image_width), dtype=f32, device=dev)
        g_image = g_image.contiguous()
        g_alpha = None if g_alpha is None else g_alpha.contiguous()
        g_depth = None if g_depth is None else g_depth.contiguous()
        image, alpha, depth = _blend_outputs(outputs)
        # one partial per (slot, cell of the batch) -- per slot at the default
        # tile, whose cells are combined on chip; only replayed entries write
        # theirs and set its flag.  Other tiles' cells run in batches of
        # fr.groups (one batch unless the partials would exceed
        # PARTIAL_BUDGET_BYTES), each summed by gs_gather_partials in order.
        G, Q = fr.groups, cam.cells
        pair_grads = torch.empty((fr.T * G, N.GS_PARTIAL_STRIDE), dtype=f32, device=dev)
        slot_live = fr.slot_live  # (zeroed by the forward's gs_tile_ranges)
        if slot_live is None:
            slot_live = torch.zeros((fr.T * G,), dtype=torch.uint8, device=dev)
        elif fr.consumed:
            # a second backward of the frame (retain_graph): the flags hold the
            # last batch's, in that batch's layout
            slot_live.zero_()
        fr.consumed = True
        ba = N.GsBlendBwdArgs(cs, cam.tiles_x, cam.tiles_y, N.ptr(fr.ranges), N.ptr(fr.sorted_gauss),
                              N.ptr(fr.records), N.ptr(image), N.ptr(alpha), N.ptr(depth),
                              N.ptr(fr.pix_flags), N.ptr(fr.cell_neval), N.ptr(g_image), N.ptr(g_alpha), N.ptr(g_depth), N.ptr(fr.live_bits),
                              0 if fr.live_bits is None else fr.live_bits.shape[1], N.ptr(pair_grads),
                              N.ptr(slot_live), fr.T, 0, 0)
        if G < cam.groups:
            batch_sums = torch.empty((n, N.GS_PAIR_GRAD_FLOATS), dtype=f32, device=dev)
            ga = N.GsProjectBwdArgs()
            ga.g.n = n
            ga.vis, ga.rects, ga.pair_offset = N.ptr(fr.vis), N.ptr(fr.rects), N.ptr(fr.pair_offset)
            ga.pair_grads, ga.slot_live, ga.grad_sums = N.ptr(pair_grads), N.ptr(slot_live), N.ptr(batch_sums)
            for b, c0 in enumerate(range(0, Q, G)):
                ba.cell_begin, ba.cell_count = c0, min(G, Q - c0)
                ga.partial_groups = ba.cell_count
                if b:
                    slot_live.zero_()
                N.check(lib.gs_blend_backward(C.byref(ba), s), "gs_blend_backward")
                N.check(lib.gs_gather_partials(C.byref(ga), 1 if b else 0, s), "gs_gather_partials")
        else:
            StageTimer.mark("blend_bwd")
            N.check(lib.gs_blend_backward(C.byref(ba), s), "gs_blend_backward")
    raw = cov3d is None
    out = dict(out or {})
    rows_ready = out.pop("_rows_ready", None)
    chunks = int(out.pop("_chunks", 1)) if rows_ready is not None else 1

    def buf(name, shape):
        t = out.get(name)
        return t.view(shape) if t is not None else torch.empty(shape, dtype=f32, device=dev)
    d_xyz = buf("xyz", (n, 3))
    d_cov = None if raw else torch.empty((n, 3, 3), dtype=f32, device=dev)
    d_scl = buf("scaling", (n, 3)) if raw else None
    d_rot = buf("rotation", (n, 4)) if raw else None
    d_col = buf("color", (n, 3))
    d_op = buf("opacity", (n,))
    gm = None if g_means2d is None else g_means2d.contiguous()
    gc = None if g_conics is None else g_conics.contiguous()
    d_sh = buf("sh_rest", (n, N.GS_SH_REST, 3)) if sh_degree > 0 else None
    gst = _gaussians_struct(n, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit, sh_rest, sh_degree)
    if pair_grads is not None and fr.groups < cam.groups:
        grad_sums, pair_grads, slot_live = batch_sums, None, None  # (summed batch by batch above)
    else:
        grad_sums = None if pair_grads is None else torch.empty((n, N.GS_PAIR_GRAD_FLOATS), dtype=f32, device=dev)
    pb = N.GsProjectBwdArgs(cs, gst, N.ptr(means2d), N.ptr(conics), N.ptr(fr.vis), N.ptr(fr.rects),
                            # Gaussian order (order=NULL): inputs/outputs stream; walking in depth
                            # order coalesces the slot reads but scatters 10 arrays (measured 2.4x slower)
                            N.ptr(fr.pair_offset), None, N.ptr(pair_grads), N.ptr(gm), N.ptr(gc), N.ptr(d_xyz),
                            N.ptr(d_cov), N.ptr(d_scl), N.ptr(d_rot), N.ptr(d_col), N.ptr(d_op), N.ptr(d_sh),
                            N.ptr(slot_live), N.ptr(grad_sums), fr.groups)
    StageTimer.mark("project_bwd")
    bounds = [n * k // chunks for k in range(chunks + 1)]
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        part = pb if (lo, hi) == (0, n) else _rows_of(pb, lo, hi)
        N.check(lib.gs_project_backward(C.byref(part), s), "gs_project_backward")
        if rows_ready is not None:
            rows_ready(lo, hi)
    StageTimer.mark("~end_bwd")
    return d_xyz, d_cov, d_scl, d_rot, d_col, d_op, d_sh


def _blend_outputs(outputs):
    """The forward's image, alpha, depth as the blend backward reads them
    (fp32, contiguous, as rasterize returned them)."""
    if outputs is None:
        raise ValueError("the blend backward needs the forward's (image, alpha, depth)")
    image, alpha, depth = outputs
    for t in (image, alpha, depth):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("the forward's image / alpha / depth must be the contiguous fp32 tensors it returned")
    return image, alpha, depth


def _backward_frame(cam: CameraParams, fr: _FastFrame, xyz, cov3d, scaling, rotation, logits, opacity, means2d,
                    conics, g_image, g_alpha, g_depth, g_means2d, g_conics, opacity_is_logit, sh_rest, sh_degree, out,
                    outputs):
    """backward_pipeline through gs_render_backward (the frame of
    _forward_frame): the blend backward and the gather in the library, then
    the projection backward -- there too unless the data-parallel reduction
    wants the rows in ranges."""
    lib = N.load()
    dev = xyz.device
    n = int(xyz.shape[0])
    f32 = torch.float32
    s = _stream()
    pixel_grads = g_image is not None or g_alpha is not None or g_depth is not None
    ba = N.GsRenderBwdArgs()
    fa = fr.fa
    ba.cam, ba.fb, ba.M, ba.T, ba.tile_alt = fa.cam, fa.fb, fr.M, fr.T, fa.tile_alt
    # (the forward's Gaussians: the tensors autograd saved for this backward)
    ba.g, ba.means2d, ba.conics, ba.vis = fa.g, fa.means2d, fa.conics, fa.vis
    pair_grads = None
    if fr.M > 0 and fr.T > 0 and pixel_grads:
        if g_image is None:
            g_image = torch.zeros((3, cam.image_height, cam.image_width), dtype=f32, device=dev)
        g_image = g_image.contiguous()
        g_alpha = None if g_alpha is None else g_alpha.contiguous()
        g_depth = None if g_depth is None else g_depth.contiguous()
        pair_grads = torch.empty((fr.T * fr.groups, N.GS_PARTIAL_STRIDE), dtype=f32, device=dev)
        image, alpha, depth = _blend_outputs(outputs)
        ba.image, ba.alpha, ba.depth = image.data_ptr(), alpha.data_ptr(), depth.data_ptr()
        ba.g_image, ba.g_alpha, ba.g_depth = N.ptr(g_image), N.ptr(g_alpha), N.ptr(g_depth)
        ba.pair_grads = pair_grads.data_ptr()
        ba.flags_zeroed = 1 if fr.slot_live_zeroed else 0
        fr.slot_live_zeroed = False  # (a second backward of the frame clears its flags first: ADVICE r05)
    gm = None if g_means2d is None else g_means2d.contiguous()
    gc = None if g_conics is None else g_conics.contiguous()
    ba.g_means2d, ba.g_conics = N.ptr(gm), N.ptr(gc)
    raw = cov3d is None
    out = dict(out or {})
    rows_ready = out.pop("_rows_ready", None)
    chunks = int(out.pop("_chunks", 1)) if rows_ready is not None else 1

    def buf(name, shape):
        t = out.get(name)
        return t.view(shape) if t is not None else torch.empty(shape, dtype=f32, device=dev)
    d_xyz = buf("xyz", (n, 3))
    d_cov = None if raw else torch.empty((n, 3, 3), dtype=f32, device=dev)
    d_scl = buf("scaling", (n, 3)) if raw else None
    d_rot = buf("rotation", (n, 4)) if raw else None
    d_col = buf("color", (n, 3))
    d_op = buf("opacity", (n,))
    d_sh = buf("sh_rest", (n, N.GS_SH_REST, 3)) if sh_degree > 0 else None
    ba.d_xyz, ba.d_cov3d, ba.d_scaling, ba.d_rotation = N.ptr(d_xyz), N.ptr(d_cov), N.ptr(d_scl), N.ptr(d_rot)
    ba.d_color_logits, ba.d_opacity, ba.d_sh_rest = N.ptr(d_col), N.ptr(d_op), N.ptr(d_sh)
    ba.project = 1 if chunks == 1 else 0
    ev = StageTimer.pair("blend_bwd")
    if ev is not None:
        ba.blend_events[0], ba.blend_events[1] = ev[0].handle, ev[1].handle
    N.check(lib.gs_render_backward(C.byref(ba), s), "gs_render_backward")
    if chunks == 1:
        if rows_ready is not None:
            rows_ready(0, n)
        return d_xyz, d_cov, d_scl, d_rot, d_col, d_op, d_sh
    # the projection backward per row range, each range's reduction issued
    # as soon as its rows are queued
    fo = fr._o()[0]
    fws = fr.frame_ws.data_ptr()
    pb = N.GsProjectBwdArgs(fa.cam, ba.g, N.ptr(means2d), N.ptr(conics), fa.vis, fws + fo[1], fws + fo[8], None,
                            None, N.ptr(gm),
                            N.ptr(gc), N.ptr(d_xyz), N.ptr(d_cov), N.ptr(d_scl), N.ptr(d_rot), N.ptr(d_col),
                            N.ptr(d_op), N.ptr(d_sh), None, ba.grad_sums if pair_grads is not None else None, 0)
    bounds = [n * k // chunks for k in range(chunks + 1)]
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        N.check(lib.gs_project_backward(C.byref(_rows_of(pb, lo, hi)), s), "gs_project_backward")
        rows_ready(lo, hi)
    return d_xyz, d_cov, d_scl, d_rot, d_col, d_op, d_sh


def _rows_of(pb: "N.GsProjectBwdArgs", lo: int, hi: int) -> "N.GsProjectBwdArgs":
    """The projection backward's arguments restricted to Gaussians [lo, hi):
    every per-Gaussian pointer advanced by lo rows (the slot partials are
    addressed through pair_offset, absolute, and stay)."""
    r = N.GsProjectBwdArgs.from_buffer_copy(pb)
    g = r.g

    def adv(ptr, row_bytes):
        return ptr + lo * row_bytes if ptr else ptr
    g.n = hi - lo
    g.xyz = adv(g.xyz, 4 * g.xyz_stride)
    g.cov3d = adv(g.cov3d, 36)
    g.scaling = adv(g.scaling, 12)
    g.rotation = adv(g.rotation, 16)
    g.color_logits = adv(g.color_logits, 4 * g.color_stride)
    g.opacity = adv(g.opacity, 4 * g.opacity_stride)
    g.sh_rest = adv(g.sh_rest, 4 * g.sh_rest_stride)
    for name, rb in (("means2d", 8), ("conics", 16), ("vis", 1), ("rects", 8), ("pair_offset", 4),
                     ("g_means2d", 8), ("g_conics", 16), ("d_xyz", 12), ("d_cov3d", 36), ("d_scaling", 12),
                     ("d_rotation", 16), ("d_color_logits", 12), ("d_opacity", 4),
                     ("d_sh_rest", 4 * N.GS_SH_REST * 3), ("grad_sums", 4 * N.GS_PAIR_GRAD_FLOATS)):
        setattr(r, name, adv(getattr(r, name), rb))
    if r.order:
        raise ValueError("row ranges need the Gaussian-order walk (order = NULL)")
    return r


class RasterizeGaussians(torch.autograd.Function):
    """Differentiable render: inputs are the model accessors' tensors, outputs
    are (image, alpha, depth, viewspace_points, conics, radii, visibility)."""

    @staticmethod
    def forward(ctx, xyz, cov3d, scaling, rotation, logits, opacity, sh_rest, cam: CameraParams,
                opacity_is_logit=False, sh_degree=0, grad_dest=None):
        image, alpha, depth, means2d, conics, radii, vis, fr = forward_pipeline(
            cam, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit, sh_rest, sh_degree,
            need_grad=_FUSE_FLAGS and any(ctx.needs_input_grad[:7]))
        ctx.cam, ctx.frame, ctx.opacity_is_logit, ctx.sh_degree = cam, fr, opacity_is_logit, sh_degree
        ctx.grad_dest = grad_dest
        # (the outputs image / alpha / depth too: the blend backward's per-pixel
        # state; autograd refuses the backward if they were modified in place)
        ctx.save_for_backward(xyz, cov3d, scaling, rotation, logits, opacity, sh_rest, means2d, conics, image, alpha,
                              depth)
        ctx.mark_non_differentiable(radii, vis)
        ctx.set_materialize_grads(False)
        return image, alpha, depth, means2d, conics, radii, vis

    @staticmethod
    def backward(ctx, g_image, g_alpha, g_depth, g_means2d, g_conics, _g_radii, _g_vis):
        xyz, cov3d, scaling, rotation, logits, opacity, sh_rest, means2d, conics, image, alpha, depth = ctx.saved_tensors
        g_conics = None if g_conics is None else g_conics.reshape(-1, 4)
        dest = ctx.grad_dest() if ctx.grad_dest is not None else None
        d_xyz, d_cov, d_scl, d_rot, d_col, d_op, d_sh = backward_pipeline(
            ctx.cam, ctx.frame, xyz, cov3d, scaling, rotation, logits, opacity, means2d, conics,
            g_image, None if g_alpha is None else g_alpha, g_depth, g_means2d, g_conics, ctx.opacity_is_logit,
            sh_rest, ctx.sh_degree, out=dest, outputs=(image, alpha, depth))
        need = ctx.needs_input_grad
        return (d_xyz if need[0] else None,
                d_cov if (cov3d is not None and need[1]) else None,
                d_scl if (scaling is not None and need[2]) else None,
                d_rot if (rotation is not None and need[3]) else None,
                d_col.view(logits.shape) if need[4] else None,
                d_op.view(opacity.shape) if need[5] else None,
                d_sh if (sh_rest is not None and need[6]) else None,
                None, None, None, None)


def rasterize(cam: CameraParams, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit=False,
              sh_rest=None, sh_degree=0, grad_dest=None):
    """opacity_is_logit: opacity holds the model's raw _opacity and the kernels
    apply get_opacity's sigmoid (fused; its gradient goes to the logit).
    sh_degree > 0: view-dependent colour from sh_rest ([N,15,3] rest
    coefficients, e.g. get_features[:,1:,:]); 0 is the reference's DC-only
    colour (include/gsplat_mi355x.h, gs_gaussians).
    grad_dest: optional callable, asked at backward time, returning None or
    {name: tensor} buffers the gradient kernels write into (names xyz,
    scaling, rotation, color, opacity, sh_rest; see backward_pipeline)."""
    _check_inputs(xyz)
    n = int(xyz.shape[0]) if xyz.dim() == 2 else -1
    if n < 0 or xyz.shape[1] != 3:
        raise ValueError(f"xyz must be [N, 3], got {tuple(xyz.shape)}")

    def prep(name, t, tail):
        """Same device as xyz, N rows of `tail` trailing shape, fp32 (other
        float dtypes are cast, the cast on the autograd tape): the kernels read
        raw fp32 rows, so anything else would be read as garbage."""
        if t is None:
            return None
        if t.device != xyz.device:
            raise RuntimeError(f"{name} is on {t.device}, the Gaussians' xyz on {xyz.device}")
        if not t.is_floating_point():
            raise TypeError(f"{name} must be a floating-point tensor, got {t.dtype}")
        if t.dim() == 0 or t.shape[0] != n or t.numel() != n * math.prod(tail):
            raise ValueError(f"{name} must hold {list(tail)} per Gaussian for N = {n}, got {tuple(t.shape)}")
        return t if t.dtype == torch.float32 else t.float()

    xyz = prep("xyz", xyz, (3,))
    cov3d = prep("cov3d", cov3d, (3, 3))
    scaling = prep("scaling", scaling, (3,))
    rotation = prep("rotation", rotation, (4,))
    logits = prep("colour", logits, (3,))
    opacity = prep("opacity", opacity, (1,))
    if cov3d is None and (scaling is None or rotation is None):
        raise ValueError("need a covariance or scaling + rotation")
    sh_degree = int(sh_degree)
    if not 0 <= sh_degree <= 3:
        raise ValueError(f"sh_degree must be in 0..3, got {sh_degree}")
    if sh_degree > 0:
        if sh_rest is None or tuple(sh_rest.shape[1:]) != (N.GS_SH_REST, 3):
            raise ValueError("sh_degree > 0 needs sh_rest of shape [N, 15, 3]")
        sh_rest = prep("sh_rest", sh_rest, (N.GS_SH_REST, 3))
        if sh_rest.stride(2) != 1 or sh_rest.stride(1) != 3:
            sh_rest = sh_rest.contiguous()
    else:
        sh_rest = None
    if cov3d is not None:
        cov3d = cov3d.reshape(-1, 3, 3)
        if not cov3d.is_contiguous():
            cov3d = cov3d.contiguous()
    else:
        scaling = scaling.contiguous()
        rotation = rotation.contiguous()
    xyz, _ = _rows(xyz, 3)
    logits, _ = _rows(logits, 3)
    opacity, _ = _rows(opacity, 1)
    return RasterizeGaussians.apply(xyz, cov3d, scaling, rotation, logits, opacity, sh_rest, cam,
                                    bool(opacity_is_logit), sh_degree, grad_dest)
