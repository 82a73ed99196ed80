"""Builds libgsplat_mi355x.so in-tree with hipcc for gfx950.

    python mini-3d-gaussian-splatting_amd/build.py [--force]

The built .so is git-ignored but travels to the GPU box with the repo
snapshot (it is not in .gpurunignore).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = [os.path.join(HERE, "csrc", n) for n in ("gsplat_mi355x.hip", "gs_loss.hip", "gs_densify.hip", "gs_render.hip")]
HDR = [os.path.join(ROOT, "include", "gsplat_mi355x.h"), os.path.join(HERE, "csrc", "gs_internal.h")]
OUT = os.path.join(HERE, "libgsplat_mi355x.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         # the blend's skip/termination decisions must replay bit-identically
         # between forward and backward, and follow the reference's unfused
         # fp32 order; no contraction of a*b+c into fma.
         "-ffp-contract=off",
         # no SLP packing of scalar fp32 math into v_pk_add/mul_f32: on gfx950
         # a packed op costs the issue time of two plain ones plus hazard nops
         # (measured: blend backward 620 -> 571 us without it)
         "-fno-slp-vectorize",
         "-Wall", "-Wno-unused-function"]


def source_hash() -> str:
    """sha256 (16 hex digits) of the library's sources and headers: names the
    build that measurements (the PMC summary) were taken on."""
    import hashlib
    h = hashlib.sha256()
    for p in SRC + HDR:
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in SRC + HDR + [__file__])


def build(force: bool = False, verbose: bool = True) -> str:
    if force or stale():
        cmd = [HIPCC, *FLAGS, "-I", os.path.join(ROOT, "include"), *SRC, "-o", OUT]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
