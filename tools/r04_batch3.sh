#!/bin/bash
# Round-4 GPU batch 3: LDS read prefetch in the blend kernels (forward: the
# next set bit's record requested before this entry's arithmetic, two
# register sets; backward phase A: entry kk + 1's staged record before entry
# kk's arithmetic), A/B against the product, then the parity tests on the
# combined build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/b3
bash tools/ab.sh 3 ab/base.so ab/fpf.so ab/bpf.so ab/fbpf.so && \
GS_LIB_PATH=$R/ab/fbpf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/b3/parity_fbpf.log 2>&1; rc=$?; tail -3 gpurun_out/b3/parity_fbpf.log; exit $rc
