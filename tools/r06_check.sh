#!/bin/bash
# Round 6 GPU pass: all GPU tests, smoke, the C3 bench (graph-replayed
# step), C2, and rocprofv3 kernel stats of a short C3 bench.
# usage: tools/r06_check.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-r06}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd "$R"
if [ "$2" != "skip-tests" ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; cat "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
fi
timeout -k 10 300 python bench.py > "$O/c3.log" 2>&1 || { echo "bench failed"; tail -30 "$O/c3.log"; exit 1; }
python - "$O/c3.log" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C3", l["value"], "ms", l["ms_per_step"], "graph", {k: l["graph"].get(k) for k in ("replayed", "nodes", "steps_redone_in_timed_region")}, "roof", l["roofline"]["avg_launch_ms"], l["roofline"]["frac"], "cpu", (l.get("cpu_baseline") or {}).get("value"))
PY
timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline > "$O/c2.log" 2>&1 || { echo "c2 bench failed"; tail -30 "$O/c2.log"; exit 1; }
python - "$O/c2.log" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C2", l["value"], "ms", l["ms_per_step"])
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --diag-steps 0 --no-cpu-baseline > "$O/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$O/prof.log"; exit 1; }
python3 "$R/tools/timed_kernel_stats.py" "$O/prof/run_kernel_trace.csv" 20 2 > "$O/kernel_stats_timed.txt" || true
tail -1 "$O/kernel_stats_timed.txt"
tail -1 "$O/prof.log" | cut -c1-300
echo done
