#!/bin/bash
# Round 3 session t: the full GPU suite + smoke, then C3 / C4 H=16 traces.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG=${TAG:-r03t}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
export NLP_TEST_REPORT_DIR=$OUT
timeout -k 10 870 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=4 > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc2=$?; tail -2 $OUT/smoke.log; echo "smoke rc=$rc2"
[ $rc -ne 0 -o $rc2 -ne 0 ] && exit 1
SPECS="${SPECS:-C3-uk-2005:JAC:16 C4-sk-2005:JAC:16}" TAG=_$TAG bash tools/gpu_r03_p4prof.sh || exit 1
exit 0
