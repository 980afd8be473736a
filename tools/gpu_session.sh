#!/bin/bash
# GPU session: STEPS (comma list, in order) out of
#   tests   -- PYTEST_FILES (default: the dist and ingest GPU tests), one pytest process
#   bench   -- the default bench line (headline + work point + both CPU baselines)
#   prof    -- rocprofv3 --kernel-trace --stats of the bench without CPU baselines or sweep
#   pmc     -- FETCH_SIZE and WRITE_SIZE passes (separate runs) of that same command
#   c5prof  -- kernel trace + stats of tools/range_call.py (C5 IHub range)
#   c5pmc   -- FETCH_SIZE / WRITE_SIZE passes of that range call
#   c5      -- the range call alone (its JSON line in c5.json)
#   c5sq    -- one --pmc pass of the counters in PMC over the range call
#   sweep   -- tools/sweep.py SWEEP_ARGS
#   sweepprof -- the same under rocprofv3 --kernel-trace --stats
#   sweeppmc  -- the same under one --pmc pass of the counters in PMC
# Output in gpurun_out/$TAG.  Every GPU step has its own time limit and the
# script stops at the first failure.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-session}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
export NLP_TEST_REPORT_DIR=$OUT
STEPS=${STEPS:-tests,bench}
BENCH_ARGS=${BENCH_ARGS:-}
PROF_CMD="python3 $REPO/bench.py --steps 5 --warmup 2 --no-cpu-baseline --sweep = --wp-steps 3 --work-point ${WP:-16} $BENCH_ARGS"
C5_CMD="python3 $REPO/tools/range_call.py ${RANGE_ARGS:-}"
cd "$REPO"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; exit $rc; fi
}
for s in ${STEPS//,/ }; do
  case $s in
    tests) run tests ${TESTS_LIMIT:-600} python -u -m pytest \
             ${PYTEST_FILES:-tests/test_gpu_dist.py tests/test_gpu_ingest.py} ${PYTEST_K:+-k "$PYTEST_K"} -m gpu -x -v \
             --durations=40 --timeout 600 --timeout-method thread -p no:cacheprovider ;;
    smoke) run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench ${BENCH_LIMIT:-900} python3 bench.py $BENCH_ARGS
           grep '^{' "$OUT/bench.log" > "$OUT/bench.json" ;;
    prof) (cd /tmp && export TMPDIR=/tmp && run prof 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/prof" -o bench -- $PROF_CMD) || exit 1 ;;
    pmc) for c in FETCH_SIZE WRITE_SIZE; do
           (cd /tmp && export TMPDIR=/tmp && run pmc_$c 600 rocprofv3 --kernel-trace --pmc $c --output-format csv \
              -d "$OUT/pmc_$c" -o pmc -- $PROF_CMD) || exit 1
         done ;;
    c5prof) (cd /tmp && export TMPDIR=/tmp && run c5prof 600 rocprofv3 --kernel-trace --stats --output-format csv \
               -d "$OUT/c5prof" -o c5 -- $C5_CMD) || exit 1 ;;
    c5) run c5 600 $C5_CMD
        grep '^{' "$OUT/c5.log" > "$OUT/c5.json" ;;
    c5sq) (cd /tmp && export TMPDIR=/tmp && run c5sq 300 rocprofv3 --kernel-trace --pmc ${PMC:-SQ_WAVE_CYCLES} \
             --output-format csv -d "$OUT/c5sq" -o pmc -- $C5_CMD) || exit 1 ;;
    c5pmc) for c in FETCH_SIZE WRITE_SIZE; do
             (cd /tmp && export TMPDIR=/tmp && run c5pmc_$c 600 rocprofv3 --kernel-trace --pmc $c --output-format csv \
                -d "$OUT/c5pmc_$c" -o pmc -- $C5_CMD) || exit 1
           done ;;
    sweep) run sweep 900 python3 tools/sweep.py ${SWEEP_ARGS:-} ;;
    sweepprof) (cd /tmp && export TMPDIR=/tmp && run sweepprof 900 rocprofv3 --kernel-trace --stats --output-format csv \
                  -d "$OUT/sweepprof" -o sweep -- python3 $REPO/tools/sweep.py ${SWEEP_ARGS:-}) || exit 1 ;;
    sweeppmc) (cd /tmp && export TMPDIR=/tmp && run sweeppmc 600 rocprofv3 --kernel-trace --pmc ${PMC:-SQ_WAVE_CYCLES} \
                 --output-format csv -d "$OUT/sweeppmc" -o pmc -- python3 $REPO/tools/sweep.py ${SWEEP_ARGS:-}) || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session done"
