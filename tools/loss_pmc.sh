#!/bin/bash
# PMC passes over the fused loss kernels at 3x1080x1920 (tools/loss_bench.py),
# one rocprofv3 run per counter group.  usage: tools/loss_pmc.sh <outdir>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-include-regex 'k_loss' -d "$OUT/p$i" -o pmc --output-format csv \
    -- python3 "$R/tools/loss_bench.py" /tmp/loss_pmc.npz 1080 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done <<'GROUPS'
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM
GROUPS
echo "pmc done: $i passes"
