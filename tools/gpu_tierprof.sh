#!/bin/bash
# Path-4 parity tests, then rocprofv3 kernel traces of large-H sweep points
# with and without the bin-0 table-size tiers.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "hash or large_hub" -p no:cacheprovider > gpurun_out/pytest_hash.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_hash.log
  [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
for t in ${TIERS:-1 0}; do
  OUT="$REPO/gpurun_out/tierprof$t"; rm -rf "$OUT"; mkdir -p "$OUT"
  NLP_HASH_TIERS=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o s -- \
    python3 "$REPO/tools/sweep.py" --metrics ${METRICS:-JAC} --hubs ${HUBS:-16,64} --cpu-hubs "" --reps 2 > "$OUT/out.log" 2> "$OUT/err.log" \
    || { echo "tiers=$t failed"; exit 1; }
  cut -c1-200 "$OUT/out.log"
done
