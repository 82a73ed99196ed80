#!/bin/bash
# Round 6: bench lines for the presets with the replayed step (C1, C2 in five
# back-to-back processes for the run-to-run spread, C3, 4K), the C4 stand-in
# (7k iterations), and the world-size-8 gloo rehearsal of bench.py (eight
# processes sharing this box's one GPU): plain gloo, and GS_DP_NATIVE=force
# (RCCL refuses the duplicate device -> every rank falls back together).
# usage: tools/r06_configs.sh <tag>
set -o pipefail
tag=${1:-r06cfg}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd "$R"
line() { python3 -c "import json,sys; d=json.loads([x for x in open(sys.argv[1]).read().splitlines() if x.startswith('{')][-1]); print(sys.argv[2], d['config']['workload'][:40], d['ms_per_step'], d['value'], d.get('graph',{}).get('replayed'))" "$1" "$2"; }
for c in C1 C3 4K; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > "$O/$c.log" 2>&1 || { echo "bench $c failed"; tail -5 "$O/$c.log"; exit 1; }
  line "$O/$c.log" $c
done
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline > "$O/C2_$i.log" 2>&1 || { echo "bench C2 failed"; tail -5 "$O/C2_$i.log"; exit 1; }
  line "$O/C2_$i.log" C2_$i
done
timeout -k 10 300 python tools/train_synthetic.py > "$O/c4.log" 2>&1 || { echo "c4 failed"; tail -20 "$O/c4.log"; exit 1; }
grep it_per_s "$O/c4.log" | head -2
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 8 --dist-backend gloo --no-cpu-baseline --steps 5 --warmup 2 \
  --spinup-steps 3 --diag-steps 1 > "$O/gloo8.log" 2>&1 || { echo "gloo8 failed"; tail -30 "$O/gloo8.log"; exit 1; }
GS_DP_NATIVE=force GS_RCCL_INIT_TIMEOUT=30 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 8 --dist-backend gloo \
  --no-cpu-baseline --steps 5 --warmup 2 --spinup-steps 3 --diag-steps 1 > "$O/gloo8_force.log" 2>&1 \
  || { echo "gloo8 force failed"; tail -30 "$O/gloo8_force.log"; exit 1; }
for f in gloo8 gloo8_force; do
  python3 -c "
import json, sys
l = json.loads([x for x in open(sys.argv[1]).read().splitlines() if x.startswith('{')][-1])
print(sys.argv[2], l['n_gpus'], l['value'], l['ms_per_step'], json.dumps(l['allreduce'])[:600])" "$O/$f.log" $f
done
echo done
