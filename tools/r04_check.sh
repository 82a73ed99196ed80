#!/bin/bash
# Round-4 GPU checks in one call: the MSD-at-tile-size sort microbenchmark,
# the C4 training test with its printed line, the native-RCCL self-check at
# world size 1 (torchrun, --force-dist: the bench line's allreduce object),
# and the default bench (CPU baseline thread sweep included).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04check
mkdir -p "$O"
cd "$R"
timeout -k 10 120 ./build/sortbench > "$O/sortbench.log" 2>&1 || { echo "sortbench failed"; tail -5 "$O/sortbench.log"; exit 1; }
cat "$O/sortbench.log"
timeout -k 10 300 python -u -m pytest tests/test_c4_training_gpu.py -x -q -s --timeout 240 --timeout-method thread > "$O/c4.log" 2>&1 || { echo "c4 failed"; tail -20 "$O/c4.log"; exit 1; }
grep '"workload"' "$O/c4.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -s --timeout 240 --timeout-method thread -k "c3_full or c2_full" > "$O/c3c2.log" 2>&1 || { echo "c3/c2 failed"; grep -E "decision-forced|px out|FAIL|Error" "$O/c3c2.log" | head -40; exit 1; }
grep -E "decision-forced|out of tolerance|grad " "$O/c3c2.log"
GS_ALLREDUCE_CHUNKS=4 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 1 --steps 20 --warmup 3 --force-dist \
  --no-cpu-baseline > "$O/rccl_world1.log" 2>&1 || { echo "rccl world1 failed"; tail -20 "$O/rccl_world1.log"; exit 1; }
python3 -c "import json;l=json.loads(open('$O/rccl_world1.log').read().strip().splitlines()[-1]);print('world1 rccl', l['ms_per_step'], l['allreduce'])"
timeout -k 10 400 python bench.py > "$O/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$O/bench.log"; exit 1; }
python3 -c "import json;l=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print('bench', l['value'], l['ms_per_step']);print(json.dumps(l['cpu_baseline']))"
