"""The C-ABI library loads and exports every symbol include/gsplat_mi355x.h
declares; struct layouts of the ctypes mirror equal the C compiler's; entry
points reject bad arguments with a status + message (no GPU needed: these
return before any HIP call)."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "gsplat_mi355x.h")


def declared_functions():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:gs_status|size_t|int32_t|int64_t|void|const char \*)\s*(gs_\w+)\s*\(", src, re.M)))


def test_header_and_binding_agree(pkg):
    assert declared_functions() == sorted(pkg._native.EXPORTS)


def test_library_exports_every_declared_symbol(pkg):
    lib = pkg._native.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", pkg._native.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared_functions():
        assert re.search(r"\bT %s$" % name, out, re.M), name


def test_abi_version(pkg):
    assert pkg._native.load().gs_abi_version() == pkg._native.GS_ABI_VERSION


def test_struct_layouts_match_c(pkg, tmp_path):
    N = pkg._native
    names = ["gs_camera", "gs_gaussians", "gs_project_args", "gs_bin_args", "gs_range_args",
             "gs_blend_fwd_args", "gs_blend_bwd_args", "gs_project_bwd_args", "gs_adam_args", "gs_loss_args", "gs_densify_args",
             "gs_frame_buffers", "gs_render_fwd_args", "gs_render_bwd_args"]
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "gsplat_mi355x.h"\nint main(){' +
                   "".join('printf("%%zu\\n", sizeof(%s));' % n for n in names) + "}")
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    sizes = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    py = [C.sizeof(t) for t in (N.GsCamera, N.GsGaussians, N.GsProjectArgs, N.GsBinArgs, N.GsRangeArgs,
                                N.GsBlendFwdArgs, N.GsBlendBwdArgs, N.GsProjectBwdArgs, N.GsAdamArgs,
                                N.GsLossArgs, N.GsDensifyArgs, N.GsFrameBuffers, N.GsRenderFwdArgs, N.GsRenderBwdArgs)]
    assert sizes == py


def test_bad_arguments_are_reported(pkg):
    N = pkg._native
    lib = N.load()
    assert lib.gs_project_forward(None, None) == 1
    assert b"null" in lib.gs_last_error()
    alt = C.c_int32(0)
    assert lib.gs_radix_sort_pairs(None, None, None, None, 10, 0, 40, 0, None, 0, C.byref(alt), None) == 1
    a = N.GsProjectArgs()
    a.cam.image_width = a.cam.image_height = 8
    a.key_bits = 32
    for bad in (0, -4, 16385):  # tile_size outside [1, GS_MAX_TILE]
        a.cam.tile_size = bad
        assert lib.gs_project_forward(C.byref(a), None) == 3
    with pytest.raises(RuntimeError, match="gs_status=3"):
        N.check(lib.gs_project_forward(C.byref(a), None), "gs_project_forward")
    a.cam.tile_size = 1
    a.cam.image_width = 4097  # 4097 tiles per axis: more than the 12-bit tile coordinates
    assert lib.gs_project_forward(C.byref(a), None) == 3
    a.cam.image_width, a.cam.tile_size = 4096, 2
    a.cam.radius_max = 256.0  # 2*256+1 px over 2-px tiles: 258 tiles wide > GS_MAX_RECT_TILES
    assert lib.gs_project_forward(C.byref(a), None) == 3
    assert b"GS_MAX_RECT_TILES" in lib.gs_last_error()
    a.cam.radius_max = 254.0  # 256 tiles: accepted (n = 0, nothing to launch)
    assert lib.gs_project_forward(C.byref(a), None) == 0
    a.cam.image_width = 300  # 150 tiles in x: any radius fits
    a.cam.radius_max = 1e6
    assert lib.gs_project_forward(C.byref(a), None) == 0
    a.cam.radius_max = float("nan")
    assert lib.gs_project_forward(C.byref(a), None) == 3
    a.cam.radius_max, a.cam.radius_min = 1.0, 2.0
    assert lib.gs_project_forward(C.byref(a), None) == 3
    a.cam.radius_min = 0.01
    for bad in (0, 33):  # depth-key window bits
        a.key_bits = bad
        assert lib.gs_project_forward(C.byref(a), None) == 1


def test_loss_bad_arguments(pkg):
    N = pkg._native
    lib = N.load()
    assert lib.gs_loss_forward(None, None) == 1
    a = N.GsLossArgs(channels=3, height=8, width=8, window=10)
    assert lib.gs_loss_forward(C.byref(a), None) == 3  # even window
    a.window = 11
    assert lib.gs_loss_forward(C.byref(a), None) == 1  # null buffers
    assert b"gs_loss_forward" in lib.gs_last_error()
    assert lib.gs_loss_backward(C.byref(a), None) == 1
    assert lib.gs_loss_workspace_bytes(3, 1080, 1920) == 8 * 3 * 34 * 60  # one float2 per 32x32 tile
    assert lib.gs_loss_workspace_bytes(0, 4, 4) == 0


def test_workspace_queries(pkg):
    lib = pkg._native.load()
    assert lib.gs_radix_sort_workspace_bytes(4096 * 3) >= 4 * (256 * 3 + 256)
    assert lib.gs_bin_workspace_bytes(1) >= 4
    # 8x8 cells per tile: ceil(L/8)^2 (the liveness bitmap and partial layouts)
    assert [lib.gs_tile_quads(t) for t in (1, 8, 9, 12, 16, 24, 32, 256, 0, 257, 4096, 4097, 16384, 16385)] == \
        [1, 1, 4, 4, 4, 9, 16, 1024, 0, 1089, 262144, 263169, 2048 ** 2, 0]
    # partials per entry of a one-batch backward: one per cell at every tile size (large
    # tiles may replay their cells in batches, rasterizer.cell_batch); 0 out of range
    assert [lib.gs_partial_groups(t) for t in (1, 16, 256, 257, 4096, 0, 16385)] == [1, 4, 1024, 1089, 262144, 0, 0]
