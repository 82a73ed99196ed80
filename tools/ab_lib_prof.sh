#!/bin/bash
# Kernel times of library variants (same ABI) under the timed bench steps:
# one rocprofv3 kernel trace per GS_LIB_PATH build, --diag-steps 0 (the
# timed steps only), summarised by tools/timed_kernel_stats.py.
# usage: tools/ab_lib_prof.sh <lib.so> [<lib.so> ...]   (paths relative to the repo root)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab_lib
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  GS_LIB_PATH=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$n" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 30 --warmup 5 --diag-steps 0 --no-cpu-baseline > "$O/prof_$n.log" 2>&1 \
    || { echo "rocprof failed: $lib"; tail -5 "$O/prof_$n.log"; exit 1; }
  python3 "$R/tools/timed_kernel_stats.py" "$O/prof_$n/run_kernel_trace.csv" 30 > "$O/kernel_stats_$n.txt" || true
  echo "== $n $(python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{')][-1]); print(d['ms_per_step'])" "$O/prof_$n.log") ms/step"
  grep -E "k_bin_emit|k_radix_hist|k_bin_partials|k_radix_scatter|k_msd|k_radix_scan|k_tile_ranges" "$O/kernel_stats_$n.txt"
done
