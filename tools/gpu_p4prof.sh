#!/bin/bash
# rocprofv3 kernel stats of the hub-threshold sweep at large H (path 4 /
# path 2 territory): where a bandwidth-scale call spends its time.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/p4prof"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o sweep -- \
  python3 "$REPO/tools/sweep.py" --metrics ${METRICS:-JAC} --hubs ${HUBS:-64} --cpu-hubs "" --reps 2 \
  > "$OUT/sweep_stdout.log" 2> "$OUT/sweep_stderr.log"
rc=$?; echo "rocprof rc=$rc"; cat "$OUT/sweep_stdout.log"
exit $rc
