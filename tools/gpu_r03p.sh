#!/bin/bash
# Round 3 session p: tests, C3 traces, the default bench line and its kernel trace.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG=${TAG:-r03p}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=3 -k "${PYTEST_K:-hash_path or hash_routing}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
[ $rc -ne 0 ] && exit $rc
SPECS="${SPECS:-C3-uk-2005:JAC:16 C3-uk-2005:AA:16}" TAG=_$TAG bash tools/gpu_r03_p4prof.sh || exit 1
timeout -k 10 420 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/bench.err; exit $rc; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print({k: d[k] for k in ('ms_per_step','value','predicted','score_ms','select_ms','host_overhead_ms')})
print(d['roofline'])
print([(x['H'], round(x['ms'],3), x['path']) for x in d['hub_sweep']])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
  python3 $REPO/bench.py --steps 20 --warmup 3 --no-cpu-baseline --sweep = > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 $REPO/tools/prof_summary.py $OUT/prof/bench_kernel_trace.csv > $OUT/step_timeline.txt; cat $OUT/step_timeline.txt
exit 0
