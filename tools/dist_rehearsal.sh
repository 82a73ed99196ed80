#!/bin/bash
# RCCL path at world size 1 (torchrun, --force-dist): overlap chunk settings side
# by side (ms/step, the backward's last-stage interval, host time spent issuing
# collectives), then kernel stats of the 1- and 4-range runs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/dist
mkdir -p "$O"
i=0
for ch in 1 2 4; do
  i=$((i+1))
  GS_ALLREDUCE_CHUNKS=$ch timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $((29540 + i)) "$R/bench.py" --gpus 1 --steps 20 --warmup 3 --force-dist \
    --no-cpu-baseline > "$O/chunks$ch.log" 2>&1 || { echo "run failed: chunks=$ch"; exit 1; }
  python3 - "$O/chunks$ch.log" "$ch" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("chunks", sys.argv[2], "ms/step", l["ms_per_step"], "project_bwd", l["stages_ms"].get("project_bwd"),
      "allreduce", l.get("allreduce"))
PY
done
timeout -k 10 300 python "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$O/nodist.log" 2>&1 || exit 1
python3 -c "import json;l=json.loads(open('$O/nodist.log').read().strip().splitlines()[-1]);print('no dist ms/step', l['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
# (no launcher under the profiler: the process group comes up from the env:// variables)
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
for ch in 1 4; do
  export MASTER_PORT=$((29560 + ch)) GS_ALLREDUCE_CHUNKS=$ch
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof$ch" -o run --output-format csv \
    -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 3 --force-dist --no-cpu-baseline > "$O/prof$ch.log" 2>&1 || { echo "prof failed $ch"; exit 1; }
  python3 - "$O/prof$ch/run_kernel_stats.csv" "$ch" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for x in rows:
    n = x["Name"]
    if "nccl" in n.lower() or "rccl" in n.lower() or "adam" in n or "copy" in n.lower():
        print(sys.argv[2], f"{n[:60]:60s} {int(x['Calls']):5d} {float(x['AverageNs']) / 1000:8.1f} us")
PY
done
