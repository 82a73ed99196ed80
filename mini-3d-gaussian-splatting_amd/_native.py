"""ctypes binding of libgsplat_mi355x.so (the C ABI in include/gsplat_mi355x.h).

The shared library is built in-tree (see build.py) and is the ONLY compute
path of this package: there is no CPU or eager-PyTorch fallback.  If the
library is missing, or no HIP device is present, every entry point raises.

torch is imported before the library is opened so that the HIP runtime torch
already loaded (libamdhip64.so.7) is the one the library binds to.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (must be loaded before the HIP library)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libgsplat_mi355x.so"
# GS_LIB_PATH overrides the in-tree library (A/B runs of kernel variants)
LIB_PATH = os.environ.get("GS_LIB_PATH") or os.path.join(_HERE, LIB_NAME)

GS_DEFAULT_TILE = 16  # renderer.py:24
GS_MAX_TILE = 16384
GS_QUAD = 8  # 8x8 pixel cells per wave, ceil(tile/8)^2 per tile (gs_tile_quads)
GS_RECORD_FLOATS = 12
GS_PAIR_GRAD_FLOATS = 10
GS_PARTIAL_STRIDE = 10  # floats between partials in pair_grads (dense; gs_partial_groups per entry)
GS_NUM_COUNTERS = 8  # M, T, depth-bits min / max, frame status, T_eff (GS_NUM_COUNTERS in the header)
GS_ABI_VERSION = 21
# frame status bits (counters[4]; the pinned counters' [5]): what a device-resident
# frame could not do on the device, so its step is redone on the host path
GS_FRAME_NEED_CAPACITY, GS_FRAME_WINDOW_MISS, GS_FRAME_EMPTY = 1, 2, 4
GS_NEED_CAPACITY, GS_RETRY_FULL_KEYS = 4, 5  # gs_render_forward: what to do next (not errors)
GS_SH_REST = 15  # [15,3] rest coefficients per Gaussian (degree <= 3)

_vp = C.c_void_p


class GsCamera(C.Structure):
    _fields_ = [
        ("image_width", C.c_int32), ("image_height", C.c_int32),
        ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
        ("view", C.c_float * 12), ("radius_min", C.c_float), ("radius_max", C.c_float),
        ("bg", C.c_float * 3), ("tile_size", C.c_int32), ("campos", C.c_float * 3),
    ]


class GsGaussians(C.Structure):
    _fields_ = [
        ("n", C.c_int32), ("xyz", _vp), ("xyz_stride", C.c_int64), ("cov3d", _vp),
        ("scaling", _vp), ("rotation", _vp), ("color_logits", _vp), ("color_stride", C.c_int64),
        ("opacity", _vp), ("opacity_stride", C.c_int64), ("opacity_is_logit", C.c_int32),
        ("sh_degree", C.c_int32), ("sh_rest", _vp), ("sh_rest_stride", C.c_int64),
    ]


class GsProjectArgs(C.Structure):
    _fields_ = [
        ("cam", GsCamera), ("g", GsGaussians), ("means2d", _vp), ("conics", _vp), ("radii", _vp),
        ("vis", _vp), ("records", _vp), ("rects", _vp), ("depth_keys", _vp),
        ("key_base", C.c_uint32), ("key_bits", C.c_int32), ("key_minmax", _vp),
    ]


class GsBinArgs(C.Structure):
    _fields_ = [
        ("n", C.c_int32), ("tiles_x", C.c_int32), ("tiles_y", C.c_int32), ("sorted_ids", _vp),
        ("rects", _vp), ("vis", _vp), ("counters", _vp), ("key_minmax", _vp), ("workspace", _vp),
        ("workspace_bytes", C.c_size_t),
        ("tile_keys", _vp), ("pair_gauss", _vp), ("pair_offset", _vp), ("records", _vp),
        ("capacity", C.c_int64), ("host_counters", _vp), ("host_seq", C.c_uint32),
        ("key_base", C.c_uint32), ("key_bits", C.c_int32), ("step_flags", _vp), ("device_counts", C.c_int32),
        ("frame_seq", _vp),
    ]


class GsRangeArgs(C.Structure):
    _fields_ = [
        ("num_pairs", C.c_int32), ("num_tiles", C.c_int32), ("sorted_keys", _vp), ("ranges", _vp),
        ("slot_live", _vp), ("cells", C.c_int32), ("num_pairs_dev", _vp),
    ]


class GsBlendFwdArgs(C.Structure):
    _fields_ = [
        ("cam", GsCamera), ("tiles_x", C.c_int32), ("tiles_y", C.c_int32), ("ranges", _vp),
        ("sorted_gauss", _vp), ("records", _vp), ("image", _vp), ("alpha", _vp), ("depth", _vp),
        ("pix_flags", _vp), ("cell_neval", _vp), ("live_bits", _vp), ("live_words", C.c_int64),
        ("pair_counts", _vp), ("num_pairs", C.c_int32), ("pix_neval", _vp),
    ]


class GsBlendBwdArgs(C.Structure):
    _fields_ = [
        ("cam", GsCamera), ("tiles_x", C.c_int32), ("tiles_y", C.c_int32), ("ranges", _vp),
        ("sorted_gauss", _vp), ("records", _vp), ("image", _vp), ("alpha", _vp), ("depth", _vp),
        ("pix_flags", _vp), ("cell_neval", _vp), ("g_image", _vp), ("g_alpha", _vp), ("g_depth", _vp),
        ("live_bits", _vp), ("live_words", C.c_int64), ("pair_grads", _vp), ("slot_live", _vp),
        ("num_pairs", C.c_int32), ("cell_begin", C.c_int32), ("cell_count", C.c_int32),
    ]


class GsProjectBwdArgs(C.Structure):
    _fields_ = [
        ("cam", GsCamera), ("g", GsGaussians), ("means2d", _vp), ("conics", _vp), ("vis", _vp),
        ("rects", _vp), ("pair_offset", _vp), ("order", _vp), ("pair_grads", _vp), ("g_means2d", _vp),
        ("g_conics", _vp), ("d_xyz", _vp), ("d_cov3d", _vp), ("d_scaling", _vp),
        ("d_rotation", _vp), ("d_color_logits", _vp), ("d_opacity", _vp), ("d_sh_rest", _vp),
        ("slot_live", _vp), ("grad_sums", _vp), ("partial_groups", C.c_int32),
    ]


class GsFrameBuffers(C.Structure):
    _fields_ = [
        ("frame_ws", _vp), ("frame_ws_bytes", C.c_size_t), ("tile_ws", _vp), ("tile_ws_bytes", C.c_size_t),
        ("capacity", C.c_int64), ("live_cells", C.c_int32), ("flag_groups", C.c_int32),
    ]


class GsRenderFwdArgs(C.Structure):
    _fields_ = [
        ("cam", GsCamera), ("g", GsGaussians), ("means2d", _vp), ("conics", _vp), ("radii", _vp), ("vis", _vp),
        ("image", _vp), ("alpha", _vp), ("depth", _vp), ("fb", GsFrameBuffers), ("key_base", C.c_uint32),
        ("key_bits", C.c_int32), ("depth_sort_msd", C.c_int32), ("zero_slot_flags", C.c_int32),
        ("host_counters_dev", _vp), ("host_counters_host", _vp), ("host_seq", C.c_uint32), ("pair_counts", _vp),
        ("pix_neval", _vp), ("resume", C.c_int32), ("poll_timeout_ms", C.c_int32), ("device_counts", C.c_int32),
        ("step_flags", _vp), ("frame_seq", _vp), ("M", C.c_int32), ("T", C.c_int32),
        ("depth_min_bits", C.c_uint32), ("depth_max_bits", C.c_uint32), ("depth_alt", C.c_int32),
        ("tile_alt", C.c_int32),
    ]


class GsRenderBwdArgs(C.Structure):
    _fields_ = [
        ("cam", GsCamera), ("g", GsGaussians), ("fb", GsFrameBuffers), ("M", C.c_int32), ("T", C.c_int32),
        ("tile_alt", C.c_int32), ("means2d", _vp), ("conics", _vp), ("vis", _vp), ("image", _vp),
        ("alpha", _vp), ("depth", _vp), ("g_image", _vp), ("g_alpha", _vp), ("g_depth", _vp), ("g_means2d", _vp), ("g_conics", _vp), ("pair_grads", _vp),
        ("flags_zeroed", C.c_int32), ("project", C.c_int32), ("d_xyz", _vp), ("d_cov3d", _vp),
        ("d_scaling", _vp), ("d_rotation", _vp), ("d_color_logits", _vp), ("d_opacity", _vp), ("d_sh_rest", _vp),
        ("grad_sums", _vp), ("blend_events", _vp * 2), ("device_counts", C.c_int32), ("fused_adam", _vp),
    ]


GS_ADAM_MAX_TENSORS = 8


class GsAdamTensor(C.Structure):
    _fields_ = [
        ("param", _vp), ("exp_avg", _vp), ("exp_avg_sq", _vp), ("grad", _vp), ("numel", C.c_int64),
        ("lr", C.c_float), ("bias_correction1", C.c_float), ("bias_correction2_sqrt", C.c_float),
        ("param_out", _vp),
    ]


class GsAdamArgs(C.Structure):
    _fields_ = [
        ("num_tensors", C.c_int32), ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float),
        ("t", GsAdamTensor * GS_ADAM_MAX_TENSORS), ("skip_flag", _vp), ("hyper", _vp), ("hyper_row", _vp),
    ]


GS_LOSS_MAX_WINDOW = 11


class GsLossArgs(C.Structure):
    _fields_ = [
        ("channels", C.c_int32), ("height", C.c_int32), ("width", C.c_int32), ("pred", _vp), ("target", _vp),
        ("lambda_dssim", C.c_float), ("window", C.c_int32), ("c1", C.c_float), ("c2", C.c_float),
        ("workspace", _vp), ("workspace_bytes", C.c_size_t), ("maps", _vp), ("out", _vp), ("g_total", _vp),
        ("d_pred", _vp),
    ]


GS_DENSIFY_SPLIT, GS_DENSIFY_CLONE, GS_DENSIFY_PRUNE = 1, 2, 4


class GsModelArrays(C.Structure):
    _fields_ = [("xyz", _vp), ("features_dc", _vp), ("features_rest", _vp), ("scaling", _vp),
                ("rotation", _vp), ("opacity", _vp)]


class GsDensifyArgs(C.Structure):
    _fields_ = [
        ("n", C.c_int32), ("rest_floats", C.c_int32), ("in_", GsModelArrays), ("xyz_grad", _vp),
        ("grad_threshold", C.c_float), ("scene_extent", C.c_float), ("split_size", C.c_float),
        ("clone_size", C.c_float), ("min_opacity", C.c_float), ("flags", C.c_int32), ("seed", C.c_uint64),
        ("adam_m_in", GsModelArrays), ("adam_v_in", GsModelArrays), ("workspace", _vp),
        ("workspace_bytes", C.c_size_t), ("counters", _vp), ("out", GsModelArrays),
        ("adam_m_out", GsModelArrays), ("adam_v_out", GsModelArrays),
    ]


# Every symbol the header declares (checked by tests/test_abi.py).
EXPORTS = (
    "gs_abi_version", "gs_last_error", "gs_project_forward", "gs_radix_sort_workspace_bytes",
    "gs_radix_sort_pairs", "gs_depth_sort_msd", "gs_bin_workspace_bytes", "gs_bin_count", "gs_bin_emit",
    "gs_tile_ranges", "gs_blend_live_words", "gs_tile_quads", "gs_partial_groups", "gs_blend_forward", "gs_blend_backward", "gs_project_backward",
    "gs_blend_backward_groups", "gs_blend_backward_lane_stats", "gs_gather_partials", "gs_frame_workspace_bytes", "gs_tile_workspace_bytes", "gs_render_forward",
    "gs_render_backward", "gs_frame_offsets", "gs_tile_offsets", "gs_adam_step", "gs_project_backward_adam", "gs_loss_workspace_bytes", "gs_loss_forward", "gs_loss_backward",
    "gs_densify_workspace_bytes", "gs_densify_count", "gs_densify_emit",
)

_lib = None
_lock = threading.Lock()


class NativeLibraryError(RuntimeError):
    pass


def _declare(lib):
    P = C.POINTER
    lib.gs_abi_version.restype = C.c_int32
    lib.gs_last_error.restype = C.c_char_p
    lib.gs_project_forward.argtypes = [P(GsProjectArgs), _vp]
    lib.gs_radix_sort_workspace_bytes.argtypes = [C.c_int32]
    lib.gs_radix_sort_workspace_bytes.restype = C.c_size_t
    lib.gs_radix_sort_pairs.argtypes = [_vp, _vp, _vp, _vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                        _vp, C.c_size_t, P(C.c_int32), _vp]
    lib.gs_depth_sort_msd.argtypes = [_vp, _vp, _vp, _vp, C.c_int32, C.c_int32, _vp, C.c_size_t, _vp,
                                      P(C.c_int32), _vp]
    lib.gs_bin_workspace_bytes.argtypes = [C.c_int32]
    lib.gs_bin_workspace_bytes.restype = C.c_size_t
    lib.gs_bin_count.argtypes = [P(GsBinArgs), _vp]
    lib.gs_bin_emit.argtypes = [P(GsBinArgs), _vp]
    lib.gs_tile_ranges.argtypes = [P(GsRangeArgs), _vp]
    lib.gs_blend_live_words.argtypes = [C.c_int32, C.c_int32]
    lib.gs_blend_live_words.restype = C.c_size_t
    lib.gs_tile_quads.argtypes = [C.c_int32]
    lib.gs_tile_quads.restype = C.c_int32
    lib.gs_partial_groups.argtypes = [C.c_int32]
    lib.gs_partial_groups.restype = C.c_int32
    lib.gs_blend_forward.argtypes = [P(GsBlendFwdArgs), _vp]
    lib.gs_blend_backward.argtypes = [P(GsBlendBwdArgs), _vp]
    lib.gs_blend_backward_groups.argtypes = [C.c_int32, C.c_int32, C.c_int32]
    lib.gs_blend_backward_groups.restype = C.c_int64
    lib.gs_blend_backward_lane_stats.argtypes = [P(GsBlendBwdArgs), _vp, _vp, _vp]
    lib.gs_project_backward.argtypes = [P(GsProjectBwdArgs), _vp]
    lib.gs_gather_partials.argtypes = [P(GsProjectBwdArgs), C.c_int32, _vp]
    lib.gs_frame_workspace_bytes.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int32]
    lib.gs_frame_workspace_bytes.restype = C.c_size_t
    lib.gs_tile_workspace_bytes.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.c_int32]
    lib.gs_tile_workspace_bytes.restype = C.c_size_t
    lib.gs_render_forward.argtypes = [P(GsRenderFwdArgs), _vp]
    lib.gs_render_backward.argtypes = [P(GsRenderBwdArgs), _vp]
    lib.gs_frame_offsets.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int32, P(C.c_size_t)]
    lib.gs_frame_offsets.restype = None
    lib.gs_tile_offsets.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.c_int32, P(C.c_size_t)]
    lib.gs_tile_offsets.restype = None
    lib.gs_adam_step.argtypes = [P(GsAdamArgs), _vp]
    lib.gs_project_backward_adam.argtypes = [P(GsProjectBwdArgs), P(GsAdamArgs), _vp]
    lib.gs_loss_workspace_bytes.argtypes = [C.c_int32, C.c_int32, C.c_int32]
    lib.gs_loss_workspace_bytes.restype = C.c_size_t
    lib.gs_loss_forward.argtypes = [P(GsLossArgs), _vp]
    lib.gs_loss_backward.argtypes = [P(GsLossArgs), _vp]
    lib.gs_densify_workspace_bytes.argtypes = [C.c_int32]
    lib.gs_densify_workspace_bytes.restype = C.c_size_t
    lib.gs_densify_count.argtypes = [P(GsDensifyArgs), _vp]
    lib.gs_densify_emit.argtypes = [P(GsDensifyArgs), _vp]
    for f in ("gs_project_forward", "gs_radix_sort_pairs", "gs_depth_sort_msd", "gs_bin_count", "gs_bin_emit",
              "gs_tile_ranges", "gs_blend_forward", "gs_blend_backward", "gs_blend_backward_lane_stats",
              "gs_project_backward", "gs_gather_partials", "gs_render_forward", "gs_render_backward", "gs_adam_step", "gs_project_backward_adam", "gs_loss_forward", "gs_loss_backward", "gs_densify_count", "gs_densify_emit"):
        getattr(lib, f).restype = C.c_int


def load(path: str = LIB_PATH):
    """Open the HIP library (no device work happens here)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise NativeLibraryError(
                    f"{LIB_NAME} not found at {path}; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
            lib = C.CDLL(path)
            _declare(lib)
            v = lib.gs_abi_version()
            if v != GS_ABI_VERSION:
                raise NativeLibraryError(f"{LIB_NAME} ABI {v} != expected {GS_ABI_VERSION}")
            _lib = lib
    return _lib


def check(status: int, what: str):
    if status != 0:
        msg = load().gs_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (gs_status={status}): {msg}")


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None) -> int:
    """The current HIP stream of `device` (default: the current device), as
    the integer handle the C ABI takes.  Through torch's raw-stream accessor:
    torch.cuda.current_stream() builds a Stream object per call (~12 us of
    host time on the box), and the render, the optimizer and every gradient
    range's collective ask for the stream."""
    if _RAW_STREAM is not None:
        if device is None or getattr(device, "index", None) is None:
            idx = torch.cuda.current_device()
        else:
            idx = device.index
        return int(_RAW_STREAM(idx))
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


_HIP = None


def _hip():
    global _HIP
    if _HIP is None:
        tl = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        _HIP = C.CDLL(tl if os.path.exists(tl) else "libamdhip64.so.7")
        _HIP.hipHostGetDevicePointer.argtypes = [C.POINTER(_vp), _vp, C.c_uint]
        _HIP.hipHostGetDevicePointer.restype = C.c_int
        _HIP.hipEventCreate.argtypes = [C.POINTER(_vp)]
        _HIP.hipEventCreate.restype = C.c_int
        _HIP.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), _vp, _vp]
        _HIP.hipEventElapsedTime.restype = C.c_int
        for name, args in (("hipStreamBeginCapture", [_vp, C.c_int]), ("hipStreamEndCapture", [_vp, C.POINTER(_vp)]),
                           ("hipGraphInstantiate", [C.POINTER(_vp), _vp, _vp, _vp, C.c_size_t]),
                           ("hipGraphLaunch", [_vp, _vp]), ("hipGraphExecDestroy", [_vp]),
                           ("hipGraphDestroy", [_vp]), ("hipGraphGetNodes", [_vp, _vp, C.POINTER(C.c_size_t)]),
                           ("hipGraphNodeGetType", [_vp, C.POINTER(C.c_int)]),
                           ("hipGraphEventRecordNodeGetEvent", [_vp, C.POINTER(_vp)]),
                           ("hipGraphExecEventRecordNodeSetEvent", [_vp, _vp, _vp]),
                           ("hipEventDestroy", [_vp]), ("hipGetErrorString", [C.c_int])):
            f = getattr(_HIP, name)
            f.argtypes = args
            f.restype = C.c_int
        _HIP.hipGetErrorString.restype = C.c_char_p
    return _HIP


def _hip_check(err: int, what: str) -> None:
    if err != 0:
        raise RuntimeError(f"{what} failed: {_hip().hipGetErrorString(err).decode(errors='replace')}")


_HIP_GRAPH_NODE_EVENT_RECORD = 7  # hipGraphNodeTypeEventRecord
_HIP_CAPTURE_THREAD_LOCAL = 1     # hipStreamCaptureModeThreadLocal


class HipGraph:
    """A HIP graph captured from the work one callable enqueues on `stream`
    (hipStreamBeginCapture / EndCapture / GraphInstantiate on the HIP runtime
    torch loaded), replayed with hipGraphLaunch.  The callable must not
    allocate or synchronise: every buffer it names is the caller's and stays
    where it is for the graph's life.  Event records the library makes during
    the capture become event record nodes (gs_render_bwd_args.blend_events);
    set_event_pair() points them at fresh events before a replay, so that
    each replay's interval can be read afterwards."""

    def __init__(self, stream: int, enqueue):
        if not stream:
            raise ValueError("HipGraph needs a non-default stream (the null stream cannot be captured)")
        h = _hip()
        self.stream, self.graph, self.exec = stream, _vp(), _vp()
        _hip_check(h.hipStreamBeginCapture(_vp(stream), _HIP_CAPTURE_THREAD_LOCAL), "hipStreamBeginCapture")
        try:
            enqueue()
        finally:
            err = h.hipStreamEndCapture(_vp(stream), C.byref(self.graph))
        _hip_check(err, "hipStreamEndCapture")
        _hip_check(h.hipGraphInstantiate(C.byref(self.exec), self.graph, None, None, 0), "hipGraphInstantiate")
        cnt = C.c_size_t(0)
        _hip_check(h.hipGraphGetNodes(self.graph, None, C.byref(cnt)), "hipGraphGetNodes")
        nodes = (_vp * max(cnt.value, 1))()
        _hip_check(h.hipGraphGetNodes(self.graph, nodes, C.byref(cnt)), "hipGraphGetNodes")
        self.num_nodes = cnt.value
        self.event_nodes = {}  # event handle recorded at capture -> its node
        for i in range(cnt.value):
            t = C.c_int(-1)
            _hip_check(h.hipGraphNodeGetType(nodes[i], C.byref(t)), "hipGraphNodeGetType")
            if t.value == _HIP_GRAPH_NODE_EVENT_RECORD:
                ev = _vp()
                _hip_check(h.hipGraphEventRecordNodeGetEvent(nodes[i], C.byref(ev)), "hipGraphEventRecordNodeGetEvent")
                self.event_nodes[ev.value] = _vp(nodes[i])

    def set_event(self, captured_event: int, event: int) -> None:
        """The node that records `captured_event` records `event` from the next replay on."""
        _hip_check(_hip().hipGraphExecEventRecordNodeSetEvent(self.exec, self.event_nodes[captured_event],
                                                              _vp(event)), "hipGraphExecEventRecordNodeSetEvent")

    def launch(self) -> None:
        _hip_check(_hip().hipGraphLaunch(self.exec, _vp(self.stream)), "hipGraphLaunch")

    def close(self) -> None:
        if self.exec:
            _hip().hipGraphExecDestroy(self.exec)
            self.exec = _vp()
        if self.graph:
            _hip().hipGraphDestroy(self.graph)
            self.graph = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RawEvent:
    """A hipEvent_t made on the HIP runtime torch loaded, for launches the
    library brackets itself (gs_render_bwd_args.blend_events): torch's Event
    objects do not know of a record made outside torch."""
    __slots__ = ("handle",)

    def __init__(self):
        h = _vp()
        if _hip().hipEventCreate(C.byref(h)) != 0:
            raise RuntimeError("hipEventCreate failed")
        self.handle = h.value

    def elapsed_ms(self, end: "RawEvent") -> float:
        ms = C.c_float(0.0)
        if _hip().hipEventElapsedTime(C.byref(ms), _vp(self.handle), _vp(end.handle)) != 0:
            raise RuntimeError("hipEventElapsedTime failed (both events recorded and complete?)")
        return float(ms.value)


def host_device_pointer(host: "torch.Tensor"):
    """The device address of a pinned host tensor (hipHostGetDevicePointer on
    the HIP runtime torch loaded), or None if the runtime does not map it --
    the caller then copies through the stream instead."""
    if not host.is_pinned():
        return None
    d = _vp()
    if _hip().hipHostGetDevicePointer(C.byref(d), _vp(host.data_ptr()), 0) != 0 or not d.value:
        return None
    return int(d.value)
