#!/bin/bash
# End-of-round pass on the final tree: GPU tests, smoke, default bench,
# rocprofv3 kernel stats, then the PMC passes whose summary bench.py reads
# (profiles/pmc_current.txt, tied to the build's source hash).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/round_check.sh r04final && bash tools/pmc_run.sh pmc_r04final && \
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r04final/bench_after_pmc.log 2>&1 && \
  python3 -c "import json;l=json.loads([x for x in open('gpurun_out/r04final/bench_after_pmc.log').read().splitlines() if x.startswith('{')][-1]);r=l['roofline'];print('bench', l['value'], l['ms_per_step'], 'traffic', r['traffic'], r['traffic_source'].get('build_match'))"
