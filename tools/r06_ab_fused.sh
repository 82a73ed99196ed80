#!/bin/bash
# A/B on one box: the replayed C3 step with the optimizer in the backward
# (--fused-adam on) against the separate Adam launch (off), alternating;
# then kernel stats of the fused build.  usage: tools/r06_ab_fused.sh <tag>
set -o pipefail
tag=${1:-r06ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd "$R"
timeout -k 10 200 python -u -m pytest tests/test_graph_step_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "tests failed"; tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for i in 1 2; do
  for m in off on; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --diag-steps 0 --fused-adam $m > "$O/c3_${m}_$i.log" 2>&1 || { echo "bench failed"; tail -20 "$O/c3_${m}_$i.log"; exit 1; }
    python -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], l['value'], l['ms_per_step'])" "$O/c3_${m}_$i.log" "$m"
  done
done
cd /tmp && export TMPDIR=/tmp
for m in off on; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$m" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --diag-steps 0 --no-cpu-baseline --fused-adam $m > "$O/prof_$m.log" 2>&1 || { echo "rocprof failed"; tail -20 "$O/prof_$m.log"; exit 1; }
python3 "$R/tools/timed_kernel_stats.py" "$O/prof_$m/run_kernel_trace.csv" 20 2 > "$O/kernel_stats_$m.txt" || true
grep -E "project_bwd|k_adam|gather|per step" "$O/kernel_stats_$m.txt"
done
cd "$R"
timeout -k 10 200 python tools/gather_order_probe.py > "$O/gather_order.log" 2>&1 || { echo "probe failed"; tail -20 "$O/gather_order.log"; exit 1; }
cat "$O/gather_order.log"
echo done
