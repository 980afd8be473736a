#!/bin/bash
# Round 3 session r: path-4 tests, C3 / C4 JAC H=16 traces, bench lines (hot stage default and exbucket).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG=${TAG:-r03r}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=3 -k "${PYTEST_K:-hash_path or random_multigraphs}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
[ $rc -ne 0 ] && exit $rc
SPECS="${SPECS:-C3-uk-2005:JAC:16 C4-sk-2005:JAC:16}" TAG=_$TAG bash tools/gpu_r03_p4prof.sh || exit 1
for hs in default 2; do
  if [ $hs = default ]; then unset NLP_HOT_STAGE; else export NLP_HOT_STAGE=$hs; fi
  timeout -k 10 420 python bench.py --no-cpu-baseline --sweep = > $OUT/bench_$hs.json 2> $OUT/bench_$hs.err
  rc=$?; echo "bench $hs rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/bench_$hs.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$hs.json'))
print({k: d[k] for k in ('ms_per_step','value','predicted','score_ms','select_ms','host_overhead_ms')})
print(d['roofline'])"
done
exit 0
