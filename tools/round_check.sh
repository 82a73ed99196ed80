#!/bin/bash
# One GPU-box pass over the current tree: gpu tests, smoke, default bench,
# rocprofv3 kernel stats of a short bench.  usage: tools/round_check.sh <tag>
set -o pipefail
tag=${1:-check}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; cat "$O/smoke.log"; exit 1; }
cat "$O/smoke.log"
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$O/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$O/prof.log"; exit 1; }
python3 "$R/tools/timed_kernel_stats.py" "$O/prof/run_kernel_trace.csv" 25 > "$O/kernel_stats_timed.txt" || true
echo done
