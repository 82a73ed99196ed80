#!/bin/bash
# A/B of environment switches on one box: alternates bench.py runs over the
# given "label:VAR=value" entries (label:- for none) and prints per-stage times.
# usage: tools/ab_env.sh <rounds> <label:VAR=value> [...]   (run from the repo root)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
rounds=$1; shift
mkdir -p "$R/gpurun_out/ab"
for ((i = 0; i < rounds; i++)); do
  for ent in "$@"; do
    n=${ent%%:*}
    kv=${ent#*:}
    if [ "$kv" = "-" ]; then envs=(); else envs=("$kv"); fi
    env "${envs[@]}" timeout -k 10 200 python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline \
      > "$R/gpurun_out/ab/${n}_$i.log" 2>&1 || { echo "bench failed: $ent"; exit 1; }
    python3 - "$R/gpurun_out/ab/${n}_$i.log" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["stages_ms"]
print(f"{sys.argv[2]:24s} ms/step {d['ms_per_step']:.4f} " + " ".join(f"{k}={v:.4f}" for k, v in s.items()), flush=True)
PY
  done
done
