#!/bin/bash
# Round 3 session u: the round-end bench + profiles first, then C3 / C4 traces,
# then path-4 tests (with the k_hp_dcls_rows8 variant) and its timing.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG=${TAG:-r03u}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
TAG=r03_final bash tools/gpu_final_bench.sh || exit 1
cd "$REPO"
SPECS="C3-uk-2005:JAC:16 C3-uk-2005:AA:16 C4-sk-2005:JAC:16" TAG=_$TAG bash tools/gpu_r03_p4prof.sh || exit 1
cd "$REPO"
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=3 -k "hash_path" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -5
[ $rc -ne 0 ] && exit $rc
NLP_HASH_ROWS8=1 SPECS="C3-uk-2005:JAC:16 C4-sk-2005:JAC:16" TAG=_${TAG}_rows8 bash tools/gpu_r03_p4prof.sh || exit 1
exit 0
