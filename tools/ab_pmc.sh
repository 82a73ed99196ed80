#!/bin/bash
# A/B of library builds with one extra PMC counter group per build:
# usage: tools/ab_pmc.sh <rounds> "<counters>" <lib.so> [<lib.so> ...]
# (bench stage times alternating over the builds, then one rocprofv3 --pmc pass
# per build over the blend kernels; per-launch means printed)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
rounds=$1; shift
ctr=$1; shift
bash "$R/tools/ab.sh" "$rounds" "$@" || exit 1
O=$R/gpurun_out/ab_pmc
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  GS_LIB_PATH=$R/$lib timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex 'k_blend' -d "$O/$n" -o pmc \
    --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --spinup-steps 2 --no-cpu-baseline > "$O/$n.log" 2>&1 \
    || { echo "pmc failed: $n"; exit 1; }
  python3 - "$O/$n/pmc_counter_collection.csv" "$n" <<'PY'
import csv, collections, re, sys
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = re.search(r"(k_\w+)", r["Kernel_Name"]).group(1)
    per[(k, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
for (k, c), d in sorted(per.items()):
    v = list(d.values())
    print(f"{sys.argv[2]:10s} {k:14s} {c:24s} {sum(v)/len(v):14.1f}")
PY
done
