#!/bin/bash
# Bench lines for the presets (C1, C2, C3, 4K), each naming its workload, plus
# a rocprofv3 kernel trace of C1 and C2 (kernel sum vs step time: host-bound?).
# usage: tools/r05_configs.sh <tag>
set -o pipefail
tag=${1:-configs}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd "$R"
for c in C1 C2 C3 4K; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > "$O/$c.log" 2>&1 || { echo "bench $c failed"; tail -5 "$O/$c.log"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['config']['workload'][:60], d['ms_per_step'], d['value'])" "$O/$c.log" $c
done
timeout -k 10 200 python tools/host_profile.py 5000 256 256 500 > "$O/hostprof_c1.log" 2>&1 || exit 1
head -3 "$O/hostprof_c1.log"
timeout -k 10 200 python tools/host_split.py 5000 256 256 500 > "$O/hostsplit_c1.log" 2>&1 || exit 1
timeout -k 10 200 python tools/host_split.py 100000 800 800 300 > "$O/hostsplit_c2.log" 2>&1 || exit 1
cat "$O/hostsplit_c1.log" "$O/hostsplit_c2.log" | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
for c in C1 C2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$c" -o run --output-format csv -- python3 "$R/bench.py" --config $c --steps 50 --warmup 5 --no-cpu-baseline > "$O/prof_$c.log" 2>&1 || { echo "rocprof $c failed"; exit 1; }
  python3 "$R/tools/timed_kernel_stats.py" "$O/prof_$c/run_kernel_trace.csv" 55 > "$O/kernel_stats_$c.txt" || true
  python3 "$R/tools/step_gpu_time.py" "$O/prof_$c/run_kernel_trace.csv" 40 | tee "$O/step_gpu_$c.txt"
done
echo done
