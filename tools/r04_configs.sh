#!/bin/bash
# Throughput of the render step (fwd + bwd + Adam) at the other configs of
# BASELINE.json (C1, C2) and at 4K, beside C3: one bench line each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/configs
mkdir -p "$O"
cd "$R"
for cfg in "c1 5000 256 256" "c2 100000 800 800" "c3 1000000 1920 1080" "uhd 4000000 3840 2160"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --gaussians $2 --width $3 --height $4 --no-cpu-baseline > "$O/$1.log" 2>&1 \
    || { echo "bench $1 failed"; tail -5 "$O/$1.log"; exit 1; }
  python3 -c "import json,sys;l=json.loads(open('$O/$1.log').read().strip().splitlines()[-1]);print('$1', l['config']['gaussians'], l['config']['width'], l['config']['height'], 'ms/step', l['ms_per_step'], 'Mpix/s', l['value'], 'T', l['config']['tile_touches'])"
done
