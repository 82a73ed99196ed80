#!/bin/bash
# A/B of the backward's gradient accumulation on one box (round-3 review item 1):
# ab/base.so (per-(entry, cell) partials + k_gather_slots) against ab/atomic.so
# (-DGS_BWD_ATOMIC=1: per-Gaussian fp32 float atomics, no gather), alternating
# bench runs, then kernel stats and WRITE_SIZE / FETCH_SIZE / TCC_EA0_ATOMIC of
# each (one rocprofv3 pass per counter group), and the C2 parity test on the atomic build.
# usage: tools/variants/ab_atomic.sh <rounds>; ab/atomic.so: patch -p1 < tools/variants/r04_atomic_accumulation.patch,
# tools/build_variant.sh atomic -DGS_BWD_ATOMIC=1, then reverse the patch (the product has no atomic path)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab_atomic
mkdir -p "$O"
rounds=${1:-3}
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$O/$n.log" 2>&1 || { echo "bench failed: $n"; tail -5 "$O/$n.log"; exit 1; }
  python3 - "$O/$n.log" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["stages_ms"]
print(f"{sys.argv[2]:14s} ms/step {d['ms_per_step']:.4f} " + " ".join(f"{k}={v:.4f}" for k, v in s.items()), flush=True)
PY
}
for ((i = 0; i < rounds; i++)); do
  run base_$i GS_LIB_PATH=$R/ab/base.so || exit 1
  run atomic_$i GS_LIB_PATH=$R/ab/atomic.so GS_BWD_ATOMIC=1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for v in base atomic; do
  ex="GS_LIB_PATH=$R/ab/$v.so"; [ $v = atomic ] && ex="$ex GS_BWD_ATOMIC=1"
  export GS_LIB_PATH=$R/ab/$v.so GS_BWD_ATOMIC=$([ $v = atomic ] && echo 1 || echo 0)
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_$v" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$O/prof_$v.log" 2>&1 || { echo "prof failed $v"; exit 1; }
  j=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_ATOMIC_sum"; do
    j=$((j+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex 'k_blend_bwd|k_gather' -d "$O/pmc_${v}_$j" -o pmc --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --spinup-steps 2 --no-cpu-baseline > "$O/pmc_${v}_$j.log" 2>&1 || { echo "pmc $v $grp failed"; exit 1; }
  done
done
unset GS_LIB_PATH GS_BWD_ATOMIC
cd "$R"
GS_LIB_PATH=$R/ab/atomic.so GS_BWD_ATOMIC=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "c2_full_size or random_scene or reference_fixture" > "$O/pytest_atomic.log" 2>&1; echo "pytest atomic rc=$?"; tail -3 "$O/pytest_atomic.log"
echo done
