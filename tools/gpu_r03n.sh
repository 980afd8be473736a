#!/bin/bash
# Round 3 session n: tests, C3 JAC H=16 trace, PMC passes of the same call.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT=$REPO/gpurun_out/${TAG:-r03n}
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=3 -k "${PYTEST_K:-hash_path or hash_routing or c3_jaccard_h16}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
[ $rc -ne 0 ] && exit $rc
SPECS="${SPECS:-C3-uk-2005:JAC:16}" TAG=_${TAG:-r03n} bash tools/gpu_r03_p4prof.sh || exit 1
SPEC=C3-uk-2005:JAC:16 TAG=${TAG:-r03n} bash tools/gpu_pmc_call.sh || exit 1
exit 0
