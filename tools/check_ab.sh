#!/bin/bash
# GPU parity of the in-tree build, then an A/B of two library builds.
# usage: tools/check_ab.sh <tag> <base.so> <new.so>   (run from the repo root on the GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
mkdir -p "$R/gpurun_out"
timeout -k 10 300 python -u -m pytest "$R/tests" -m gpu -x -q -s --timeout 120 --timeout-method thread \
  > "$R/gpurun_out/pytest_$tag.log" 2>&1
rc=$?
grep -E "C3:|passed|failed" "$R/gpurun_out/pytest_$tag.log"
[ $rc -eq 0 ] || { echo "gpu tests failed ($rc)"; exit $rc; }
"$R/tools/ab.sh" 3 "$@"
