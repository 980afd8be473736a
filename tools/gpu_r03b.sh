#!/bin/bash
# Round 3 GPU session B: the C3 / C5 / C1 full-size tests and the >2^32 test,
# then the rocprofv3 kernel trace + stats of the default bench command and its
# FETCH_SIZE / WRITE_SIZE passes.  Output in gpurun_out/r03b/.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT=$REPO/gpurun_out/r03b
mkdir -p $OUT
export NLP_TEST_REPORT_DIR=$OUT
timeout -k 10 840 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail=4 -k "${PYTEST_K:-c3 or c5 or c1 or big_offsets}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -12
case $rc in 0|1) ;; *) exit $rc ;; esac
[ -n "${SKIP_PROF:-}" ] && exit 0
cd /tmp && export TMPDIR=/tmp
B="$REPO/bench.py --steps 20 --warmup 3 --no-cpu-baseline --sweep ="
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
  python3 $B > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?; echo "rocprof rc=$rc"; cut -c1-200 $OUT/prof_bench.json; [ $rc -ne 0 ] && exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/pmc_$c -o pmc -- \
    python3 $REPO/bench.py --steps 5 --warmup 2 --no-cpu-baseline --sweep = > $OUT/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
