#!/bin/bash
# Rehearsal of the native-RCCL establishment protocol's failure path on a
# one-GPU box: two gloo ranks on the same GPU with GS_DP_NATIVE=force build
# RcclComm; RCCL refuses the duplicate device in ncclCommInitRank, and both
# ranks must agree, fall back to torch.distributed together and finish the
# bench (the line's allreduce object names the reason).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04dist
mkdir -p "$O"
cd "$R"
GS_DP_NATIVE=force timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --steps 5 --warmup 2 --spinup-steps 3 \
  --dist-backend gloo --no-cpu-baseline > "$O/force_gloo2.log" 2>&1 || { echo "force gloo2 failed"; tail -30 "$O/force_gloo2.log"; exit 1; }
grep -i "native rccl\|warn" "$O/force_gloo2.log" | head -5
python3 -c "import json;l=json.loads([x for x in open('$O/force_gloo2.log').read().splitlines() if x.startswith('{')][-1]);print('gloo2 forced native', l['ms_per_step'], l['allreduce'])"
