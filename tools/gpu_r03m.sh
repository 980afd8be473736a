#!/bin/bash
# Round 3 session m: path-4 tests, then kernel traces of C3 / C4 JAC H = 16.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT=$REPO/gpurun_out/${TAG:-r03m}
mkdir -p $OUT
if [ -z "${NO_PYTEST:-}" ]; then
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=3 -k "${PYTEST_K:-hash_path or hash_routing or random_multigraphs or c3_jaccard_h16}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
[ $rc -ne 0 ] && exit $rc
fi
SPECS="${SPECS:-C3-uk-2005:JAC:16 C4-sk-2005:JAC:16}" TAG=_${TAG:-r03m} bash tools/gpu_r03_p4prof.sh || exit 1
exit 0
