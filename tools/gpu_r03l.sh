#!/bin/bash
# Round 3 session l: path-4 / routing / C2 / C3 tests, then kernel traces of
# C3 JAC / AA at H = 16, and C2 AA H = 16 on path 4 vs the sort path.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT=$REPO/gpurun_out/${TAG:-r03l}
mkdir -p $OUT
if [ -z "${NO_PYTEST:-}" ]; then
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=3 -k "${PYTEST_K:-hash_path or hash_routing or c2_large or c3}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
[ $rc -ne 0 ] && exit $rc
fi
SPECS="${SPECS:-C3-uk-2005:JAC:16 C3-uk-2005:AA:16}" TAG=_${TAG:-r03l} bash tools/gpu_r03_p4prof.sh || exit 1
for aa in 1 0; do
  NLP_HASH_AA=$aa timeout -k 10 300 python3 tools/sweep.py --config C2-soc-LiveJournal1 --metrics AA --hubs 16 --cpu-hubs "" --reps 2 \
    > $OUT/c2_aa16_$aa.jsonl 2> $OUT/c2_aa16_$aa.err
  rc=$?; echo "c2 AA16 hash_aa=$aa rc=$rc"; cut -c1-300 $OUT/c2_aa16_$aa.jsonl
  [ $rc -ne 0 ] && exit $rc
done
exit 0
