#!/bin/bash
# Round 3 session s: path-4 tests + C3/C4 full-size path-4 tests, C3 / C4 JAC H=16 traces.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG=${TAG:-r03s}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=3 -k "${PYTEST_K:-hash_path or random_multigraphs or c3_jaccard_h16 or c3_adamic_adar_h16 or c4_jaccard_h16}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
[ $rc -ne 0 ] && exit $rc
SPECS="${SPECS:-C3-uk-2005:JAC:16 C3-uk-2005:AA:16 C4-sk-2005:JAC:16}" TAG=_$TAG bash tools/gpu_r03_p4prof.sh || exit 1
exit 0
