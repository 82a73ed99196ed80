#!/bin/bash
# RCCL path at world size 1 (torchrun, --force-dist): overlap chunk settings side by side.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/dist"
i=0
for ch in 1 2 4; do
  i=$((i+1))
  GS_ALLREDUCE_CHUNKS=$ch timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $((29540 + i)) "$R/bench.py" --gpus 1 --steps 20 --warmup 3 --force-dist \
    --no-cpu-baseline > "$R/gpurun_out/dist/chunks$ch.log" 2>&1 || { echo "run failed: chunks=$ch"; exit 1; }
  python3 - "$R/gpurun_out/dist/chunks$ch.log" "$ch" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("chunks", sys.argv[2], "ms/step", l["ms_per_step"], "project_bwd", l["stages_ms"].get("project_bwd"))
PY
done
timeout -k 10 300 python "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/dist/nodist.log" 2>&1 || exit 1
python3 -c "import json;l=json.loads(open('$R/gpurun_out/dist/nodist.log').read().strip().splitlines()[-1]);print('no dist ms/step', l['ms_per_step'])"
