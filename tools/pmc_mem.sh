#!/bin/bash
# FETCH_SIZE and WRITE_SIZE per kernel (two rocprofv3 --pmc passes) for the
# in-tree library or a variant build.  usage: tools/pmc_mem.sh <tag> [lib.so]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p "$OUT"
if [ -n "$2" ]; then export GS_LIB_PATH=$R/$2; fi
cd /tmp && export TMPDIR=/tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex 'k_' -d "$OUT/p$i" -o pmc --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --spinup-steps 2 --no-cpu-baseline > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$OUT" k_blend_bwd k_gather > "$OUT/summary.txt" && cat "$OUT/summary.txt"
