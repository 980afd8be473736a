#!/bin/bash
# Full GPU suite (pytest -m gpu) + smoke, output in gpurun_out/${TAG}.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG=${TAG:-suite}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
export NLP_TEST_REPORT_DIR=$OUT
timeout -k 10 ${SUITE_TIMEOUT:-1000} python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=4 ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc2=$?; tail -3 $OUT/smoke.log; echo "smoke rc=$rc2"
exit $(( rc | rc2 ))
