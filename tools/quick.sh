#!/bin/bash
# Quick GPU perf pass: default bench (no CPU baseline) + rocprofv3 kernel
# stats of a short bench, summarised.  usage: tools/quick.sh <tag> [bench args]
set -o pipefail
tag=${1:-quick}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$O/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$O/bench.log"; exit 1; }
python - "$O/bench.log" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", l["value"], "ms", l["ms_per_step"], "stages", l["stages_ms"])
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline "$@" > "$O/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$O/prof.log"; exit 1; }
python3 - "$O/prof/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = 0.0
for x in rows:
    us = float(x["AverageNs"]) / 1000
    if int(x["Calls"]) >= 20:
        print(f"{x['Name'][:64]:64s} {int(x['Calls']):5d} {us:8.1f} us")
PY
echo done
