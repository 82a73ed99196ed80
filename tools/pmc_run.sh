#!/bin/bash
# PMC passes (tools/pmc.sh) + summary into profiles/pmc_current.txt and gpurun_out/<tag>/pmc_summary.txt
set -o pipefail
tag=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/tools/pmc.sh" "gpurun_out/$tag" || exit 1
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/$tag" k_ > "$R/gpurun_out/$tag/pmc_summary.txt" || exit 1
cp "$R/gpurun_out/$tag/pmc_summary.txt" "$R/profiles/pmc_current.txt"
mkdir -p "$R/gpurun_out/profiles_copy" && cp "$R/profiles/pmc_current.txt" "$R/gpurun_out/profiles_copy/pmc_current.txt"
echo pmc ok
