#!/bin/bash
# Round-4 GPU batch: RCCL failure-path rehearsal, forward staging / XCD mapping
# A/B with LDS PMC, the large-tile parity tests (printed), the GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/b2
echo "(r04_dist done: profiles/r04/dist)" && \
bash tools/ab_pmc.sh 3 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU" ab/base.so ab/soa.so ab/rows.so ab/bw7.so && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -s --timeout 300 --timeout-method thread -k large_tiles > gpurun_out/b2/large_tiles.log 2>&1 && \
grep -E "tile[0-9]+|passed|failed" gpurun_out/b2/large_tiles.log | tail -40 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/b2/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/b2/pytest_gpu.log; exit $rc
