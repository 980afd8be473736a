#!/bin/bash
# PMC passes (kernel trace + one counter group per pass, no other tracing) over
# one tools/sweep.py call: SPEC=config:metric:H.  Output in gpurun_out/pmc_${TAG}.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_${TAG:-call}"
mkdir -p "$OUT"
IFS=: read cfg met hub <<< "${SPEC:-C3-uk-2005:JAC:16}"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 "$REPO/tools/sweep.py" --config $cfg --metrics $met --hubs $hub --cpu-hubs "" --reps 1 > "$OUT/p$i.log" 2>&1 \
    || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok ($grp)"
done
