#!/bin/bash
# Round 3 session: a test selection, the default bench line, its kernel trace
# (step timeline), then the large-H kernel traces.  Output in gpurun_out/${TAG}.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG=${TAG:-r03f}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
export NLP_TEST_REPORT_DIR=$OUT
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    --maxfail=4 -k "$PYTEST_K" > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
  case $rc in 0|1) ;; *) exit $rc ;; esac
fi
timeout -k 10 420 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json,sys; d=json.load(open('$OUT/bench.json'))
print({k: d[k] for k in ('ms_per_step','value','predicted','score_ms','select_ms','host_overhead_ms')})
print([(x['H'], round(x['ms'],3), x['path']) for x in d['hub_sweep']])"
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
  python3 $REPO/bench.py --steps 20 --warmup 3 --no-cpu-baseline --sweep = > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 $REPO/tools/prof_summary.py $OUT/prof/bench_kernel_trace.csv > $OUT/step_timeline.txt; cat $OUT/step_timeline.txt
[ -n "${SKIP_P4:-}" ] && exit 0
TAG=_$TAG bash $REPO/tools/gpu_r03_p4prof.sh
