#!/bin/bash
# Build a variant of the library into ab/<name>.so with extra compiler flags
# (e.g. -DGS_BWD_GROUP=4), for tools/ab.sh.  usage: tools/build_variant.sh <name> [flags...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p "$R/ab"
C=$R/mini-3d-gaussian-splatting_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize \
  -Wall -Wno-unused-function -I "$R/include" "$@" "$C/gsplat_mi355x.hip" "$C/gs_loss.hip" "$C/gs_densify.hip" "$C/gs_render.hip" \
  -o "$R/ab/$name.so"
echo "built ab/$name.so"
