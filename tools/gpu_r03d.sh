#!/bin/bash
# Round 3 session D: the new small-order / multi-device / drop-in tests, the
# default bench line, then the path-4 / path-2 kernel traces at large H.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT=$REPO/gpurun_out/r03d
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=4 -k "${PYTEST_K:-small_order or multi or dropin or cpp or survivor or async or counted}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 420 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-700 $OUT/bench.json; [ $rc -ne 0 ] && exit $rc
[ -n "${SKIP_PROF:-}" ] && exit 0
TAG=_r03d bash tools/gpu_r03_p4prof.sh
