#!/bin/bash
# Round 3 session k: path-4 tests, C3 AA H=16 on path 4 against the oracle,
# then C3 timings (JAC / AA default routes, AA on path 4).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT=$REPO/gpurun_out/${TAG:-r03k}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=3 -k "${PYTEST_K:-hash_path}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
[ $rc -ne 0 ] && exit $rc
NLP_HASH=1 timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "c3_adamic_adar_h16" > $OUT/pytest_c3aa.log 2>&1
rc=$?; echo "pytest c3 AA path 4 rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_c3aa.log | tail -12
[ $rc -ne 0 ] && exit $rc
NO_PYTEST=1 SPECS="${SPECS:-C3-uk-2005:AA:16:1 C3-uk-2005:JAC:16:0}" TAG=${TAG:-r03k} bash tools/gpu_r03j.sh
