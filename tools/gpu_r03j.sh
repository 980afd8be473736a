#!/bin/bash
# Round 3 session j: path-4 tests (optional), then C3 timings of JAC / AA at
# H = 16 on the default routes and AA forced onto path 4 (NLP_HASH=1).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG=${TAG:-r03j}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "${PYTEST_K:-}" ] && [ -z "${NO_PYTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    --maxfail=3 -k "$PYTEST_K" > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
  [ $rc -ne 0 ] && exit $rc
fi
for spec in ${SPECS:-C3-uk-2005:JAC,AA:16:0 C3-uk-2005:AA:16:1}; do
  IFS=: read cfg met hub hash <<< "$spec"
  name=${cfg%%-*}_${met/,/_}_${hub}_h${hash}
  if [ "$hash" = "1" ]; then export NLP_HASH=1; else unset NLP_HASH; fi
  timeout -k 10 400 python3 tools/sweep.py --config $cfg --metrics $met --hubs $hub --cpu-hubs "" --reps 2 \
    > $OUT/$name.jsonl 2> $OUT/$name.err
  rc=$?; echo "$name rc=$rc"; cut -c1-330 $OUT/$name.jsonl
  [ $rc -ne 0 ] && { tail -5 $OUT/$name.err; exit $rc; }
done
exit 0
