#!/bin/bash
# Round 3 GPU session A: the GPU suite without the three largest configs (C4
# and the >2^32-entry graph included), then the default bench line (C4).
# Output in gpurun_out/r03a/.  Stops at a fault / abort / time limit.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT=gpurun_out/r03a
mkdir -p $OUT
export NLP_TEST_REPORT_DIR=$REPO/$OUT
timeout -k 10 780 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=4 -k "${PYTEST_K:-not c3 and not c5 and not c1}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 420 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-1500 $OUT/bench.json; tail -3 $OUT/bench.err
exit $rc
