#!/bin/bash
# rocprofv3 kernel trace of a short bench run; prints the last step's kernel timeline.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/tl${1:-}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o bench -- \
  python3 "$REPO/bench.py" --steps ${BENCH_STEPS:-10} --warmup 3 --no-cpu-baseline > "$OUT/bench_stdout.log" 2> "$OUT/bench_stderr.log"
rc=$?; echo "rocprof rc=$rc"; tail -1 "$OUT/bench_stdout.log" | cut -c1-300
[ $rc -ne 0 ] && exit $rc
TR=$(find "$OUT" -name "*kernel_trace.csv" | head -1)
python3 "$REPO/tools/prof_summary.py" "$TR" > "$OUT/step_timeline.txt"
cat "$OUT/step_timeline.txt"
