#!/bin/bash
# C1 step time with the bench process pinned to one / two CPUs vs unpinned,
# alternating processes on one box (host-placement probe for the C1 spread).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c1pin
mkdir -p "$O"
cd "$R"
for i in 1 2 3 4; do
  for mode in none c8 c8_9; do
    case $mode in
      none) pre="" ;;
      c8) pre="taskset -c 8" ;;
      c8_9) pre="taskset -c 8,9" ;;
    esac
    timeout -k 10 120 $pre python bench.py --config C1 --no-cpu-baseline > "$O/${mode}_$i.log" 2>&1 || { echo "bench $mode failed"; tail -3 "$O/${mode}_$i.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" "$O/${mode}_$i.log" $mode
  done
done
