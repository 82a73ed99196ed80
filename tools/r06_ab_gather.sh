#!/bin/bash
# A/B of the gather variants (ab/cur.so, ab/gplain.so), alternating, kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab_gather
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for i in 1; do
for n in cur; do
  GS_LIB_PATH=$R/ab/$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_${n}_$i" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 30 --warmup 5 --diag-steps 0 --no-cpu-baseline > "$O/prof_${n}_$i.log" 2>&1 \
    || { echo "rocprof failed: $n"; tail -5 "$O/prof_${n}_$i.log"; exit 1; }
  python3 "$R/tools/timed_kernel_stats.py" "$O/prof_${n}_$i/run_kernel_trace.csv" 30 2 > "$O/kernel_stats_${n}_$i.txt" || true
  echo "== $n $i: $(grep gather "$O/kernel_stats_${n}_$i.txt") | $(tail -1 "$O/kernel_stats_${n}_$i.txt")"
done
done
