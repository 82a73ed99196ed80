#!/bin/bash
# The N > 1 bench line's all-reduce numbers on a one-GPU box (the 8-GPU run is
# the driver's): bench.py at world size 1 through the native RCCL communicator
# (--force-dist), and two gloo ranks sharing the GPU.  Prints each line's
# allreduce object (gpu_us_per_step, exposed_frac).  usage: r05_dist.sh [config]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05dist
CFG=${1:-C3}
mkdir -p "$O"
cd "$R"
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29581 timeout -k 10 300 \
  python bench.py --force-dist --config "$CFG" --no-cpu-baseline > "$O/world1_native_$CFG.log" 2>&1 \
  || { echo "world1 native failed"; tail -30 "$O/world1_native_$CFG.log"; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29582 bench.py --gpus 2 --config "$CFG" --dist-backend gloo --no-cpu-baseline \
  > "$O/gloo2_$CFG.log" 2>&1 || { echo "gloo2 failed"; tail -30 "$O/gloo2_$CFG.log"; exit 1; }
for f in "$O/world1_native_$CFG.log" "$O/gloo2_$CFG.log"; do
  python3 -c "
import json, sys
l = json.loads([x for x in open(sys.argv[1]).read().splitlines() if x.startswith('{')][-1])
print(sys.argv[1].split('/')[-1], l['value'], l['ms_per_step'], json.dumps(l['allreduce']))" "$f"
done
