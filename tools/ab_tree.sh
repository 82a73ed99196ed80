#!/bin/bash
# A/B of whole source trees on one box (for changes that move the ABI, where
# tools/ab.sh's library swap cannot run the old build): alternates bench.py
# runs from each tree (each with its own in-tree library) and prints the step
# time, the live blend-backward launch time and the diagnostic blend-forward
# time; then one rocprofv3 kernel-stats run per tree.
# usage: tools/ab_tree.sh <rounds> <tree> [<tree> ...]   (trees relative to the repo root; "." = this one)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
rounds=$1; shift
O=$R/gpurun_out/ab_tree
mkdir -p "$O"
for ((i = 0; i < rounds; i++)); do
  for t in "$@"; do
    n=$(echo "$t" | tr '/.' '__')
    (cd "$R/$t" && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline) > "$O/${n}_$i.log" 2>&1 \
      || { echo "bench failed: $t"; tail -5 "$O/${n}_$i.log"; exit 1; }
    python3 - "$O/${n}_$i.log" "$t" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]:16s} ms/step {d['ms_per_step']:.4f}  blend_bwd(live) {r['avg_launch_ms']:.4f}  "
      f"blend_fwd(diag) {r.get('other_blend', {}).get('avg_ms', float('nan')):.4f}", flush=True)
PY
  done
done
cd /tmp && export TMPDIR=/tmp
for t in "$@"; do
  n=$(echo "$t" | tr '/.' '__')
  (cd "$R/$t" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$n" -o run --output-format csv \
    -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > "$O/prof_$n.log" 2>&1) || { echo "rocprof failed: $t"; exit 1; }
  python3 "$R/tools/timed_kernel_stats.py" "$O/prof_$n/run_kernel_trace.csv" 35 > "$O/kernel_stats_$n.txt" || true
  echo "== $t"; head -8 "$O/kernel_stats_$n.txt"
done
