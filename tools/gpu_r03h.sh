#!/bin/bash
# Round 3 session h: a test selection, the default bench line (+ direct
# launches), and the path-4 bin statistics of C3 / C4 JAC H = 16
# (NLP_HASH_STATS=1).  Output in gpurun_out/${TAG}.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG=${TAG:-r03h}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    --maxfail=4 -k "$PYTEST_K" > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
  case $rc in 0|1) ;; *) exit $rc ;; esac
fi
timeout -k 10 420 python bench.py --no-cpu-baseline --sweep = > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print({k: d[k] for k in ('ms_per_step','value','predicted','score_ms','select_ms','host_overhead_ms')})"
[ $rc -ne 0 ] && exit $rc
NLP_DIRECT_LAUNCH=1 timeout -k 10 420 python bench.py --no-cpu-baseline --sweep = > $OUT/bench_direct.json 2> $OUT/bench_direct.err
rc=$?; echo "bench direct rc=$rc"; python3 -c "
import json; d=json.load(open('$OUT/bench_direct.json'))
print({k: d[k] for k in ('ms_per_step','value','predicted','score_ms','select_ms','host_overhead_ms')})"
[ $rc -ne 0 ] && exit $rc
for spec in ${SPECS:-C3-uk-2005:JAC:16 C4-sk-2005:JAC:16}; do
  IFS=: read cfg met hub <<< "$spec"
  name=${cfg%%-*}_${met}_${hub}
  NLP_HASH_STATS=1 timeout -k 10 400 python3 tools/sweep.py --config $cfg --metrics $met --hubs $hub --cpu-hubs "" --reps 1 \
    > $OUT/stats_$name.jsonl 2> $OUT/stats_$name.err
  rc=$?; echo "$name rc=$rc"; grep "hash-stats" $OUT/stats_$name.err | head -60; cut -c1-300 $OUT/stats_$name.jsonl
  [ $rc -ne 0 ] && exit $rc
done
exit 0
