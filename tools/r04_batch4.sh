#!/bin/bash
# Round-4 GPU batch 4: the native RCCL path after the bounded self-check wait
# (world-size-1 bench through torch.distributed.run, the forced two-rank
# failure-path rehearsal), the distributed GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/b4
mkdir -p "$O"
cd "$R"
GS_ALLREDUCE_CHUNKS=4 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29581 bench.py --gpus 1 --steps 20 --warmup 3 --force-dist --no-cpu-baseline \
  > "$O/rccl_world1.log" 2>&1 || { echo "rccl world1 failed"; tail -20 "$O/rccl_world1.log"; exit 1; }
python3 -c "import json;l=json.loads(open('$O/rccl_world1.log').read().strip().splitlines()[-1]);print('world1 rccl', l['ms_per_step'], l['allreduce'])" && \
bash tools/r04_dist.sh && \
timeout -k 10 400 python -u -m pytest tests/test_dp_training_gpu.py -x -q --timeout 300 --timeout-method thread > "$O/dp_tests.log" 2>&1 && tail -2 "$O/dp_tests.log" && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -s --timeout 240 --timeout-method thread -k degenerate > "$O/degenerate.log" 2>&1; rc=$?; grep -E "grad |passed|failed|Error|assert" "$O/degenerate.log" | head -30; exit $rc
