#!/bin/bash
# rocprofv3 kernel trace + stats of the bench (no PMC counters in this pass).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/prof${1:-}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o bench -- \
  python3 "$REPO/bench.py" --steps ${BENCH_STEPS:-20} --warmup 3 --no-cpu-baseline > "$OUT/bench_stdout.log" 2> "$OUT/bench_stderr.log"
rc=$?; echo "rocprof rc=$rc"; tail -1 "$OUT/bench_stdout.log"
find "$OUT" -name "*stats*" | head
exit $rc
