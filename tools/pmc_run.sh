#!/bin/bash
# PMC passes (tools/pmc.sh) + summary into profiles/pmc_current.txt and gpurun_out/<tag>/pmc_summary.txt
set -o pipefail
tag=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/tools/pmc.sh" "gpurun_out/$tag" || exit 1
# first line: the source hash of the library the counters were taken on
# (bench.py compares it with the build it benches)
{ echo "# library_source_sha256 $(python3 -c "import sys; sys.path.insert(0, '$R/mini-3d-gaussian-splatting_amd'); import build; print(build.source_hash())")"
  python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/$tag" k_; } > "$R/gpurun_out/$tag/pmc_summary.txt" || exit 1
cp "$R/gpurun_out/$tag/pmc_summary.txt" "$R/profiles/pmc_current.txt"
mkdir -p "$R/gpurun_out/profiles_copy" && cp "$R/profiles/pmc_current.txt" "$R/gpurun_out/profiles_copy/pmc_current.txt"
echo pmc ok
