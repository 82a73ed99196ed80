#!/bin/bash
# PMC summary of the current build (profiles/pmc_current.txt) and a bench line
# + kernel stats on the same box, then the roofline table from them.
set -o pipefail
tag=${1:-r06pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd "$R"
bash tools/pmc_run.sh "$tag" || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > "$O/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --diag-steps 0 --no-cpu-baseline > "$O/prof.log" 2>&1 || { echo "rocprof failed"; exit 1; }
python3 "$R/tools/timed_kernel_stats.py" "$O/prof/run_kernel_trace.csv" 20 2 > "$O/kernel_stats_timed.txt" || true
python3 "$R/tools/roofline_table.py" "$R/profiles/pmc_current.txt" "$O/kernel_stats_timed.txt" "$O/bench.log" > "$O/roofline_table.txt" || exit 1
cat "$O/roofline_table.txt"
tail -1 "$O/kernel_stats_timed.txt"
echo done
