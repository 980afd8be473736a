#!/bin/bash
# Round 3 session v: PMC passes of the bench command, path-4 tests (rows8
# variant included), C3 / C4 traces with and without rows8.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG=${TAG:-r03v}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT $REPO/gpurun_out/r03_final/pmc
cd /tmp && export TMPDIR=/tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$REPO/gpurun_out/r03_final/pmc/p$i" -o pmc -- \
    python3 "$REPO/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --sweep = > "$REPO/gpurun_out/r03_final/pmc/p$i.log" 2>&1 \
    || { echo "pmc pass $i failed"; exit 1; }
  echo "pmc pass $i ok ($grp)"
done
cd "$REPO"
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=3 -k "hash_path" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -5
[ $rc -ne 0 ] && exit $rc
SPECS="C3-uk-2005:JAC:16 C3-uk-2005:AA:16 C4-sk-2005:JAC:16" TAG=_$TAG bash tools/gpu_r03_p4prof.sh || exit 1
cd "$REPO"
NLP_HASH_ROWS8=1 SPECS="C3-uk-2005:JAC:16 C4-sk-2005:JAC:16" TAG=_${TAG}_rows8 bash tools/gpu_r03_p4prof.sh || exit 1
exit 0
