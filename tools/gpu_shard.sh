#!/bin/bash
# One-GPU rehearsal of the N-rank step (tools/shard_emul.py) for N = 2 and 8,
# then a rocprofv3 kernel trace of the 8-rank rehearsal (per-kernel timeline).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT=gpurun_out/shard
mkdir -p $OUT
for N in ${RANKS:-2 8}; do
  timeout -k 10 300 python tools/shard_emul.py --ranks $N --steps 5 > $OUT/emul$N.json 2> $OUT/emul$N.err \
    || { echo "emul $N failed"; tail -5 $OUT/emul$N.err; exit 1; }
  cut -c1-900 $OUT/emul$N.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/$OUT/prof" -o emul -- \
  python3 "$REPO/tools/shard_emul.py" --ranks 8 --steps 3 > "$REPO/$OUT/prof.log" 2>&1 || { echo "rocprof failed"; exit 1; }
python3 - "$(find "$REPO/$OUT/prof" -name '*kernel_stats.csv' | head -1)" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:28]:
    print("%6d calls %10.1f us avg %8.2f ms tot  %s" % (int(r["Calls"]), float(r["AverageNs"]) / 1e3,
          float(r["TotalDurationNs"]) / 1e6, r["Name"][:90]))
PY
