#!/bin/bash
# Per-workgroup phase stamps (NLP_STAMP) of the sort-path stages of the bench
# call: one short bench run per stage, then tools/stamps.py on each.
#   stages (one MSD pass): 4 = MSD pass, 5 = bucket sort, 6 = run scoring
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/stamps
for s in ${STAGES:-4 5 6}; do
  rm -f gpurun_out/stamps/s$s.bin
  NLP_STAMP=gpurun_out/stamps/s$s.bin NLP_HOT_STAGE=$s timeout -k 10 300 python bench.py --steps 5 --warmup 2 \
    --no-cpu-baseline > gpurun_out/stamps/s$s.log 2>&1 || { echo "stage $s failed"; exit 1; }
  echo "== stage $s"; python tools/stamps.py gpurun_out/stamps/s$s.bin 8 ${CLOCK_SLOTS:-} && rm -f gpurun_out/stamps/s$s.bin
done
