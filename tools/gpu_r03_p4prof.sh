#!/bin/bash
# Kernel trace of the large-H calls (path 4 hash accumulation, path 2 chunked
# sort) on the C3 / C4 stand-ins: tools/sweep.py under rocprofv3 --kernel-trace
# --stats.  Output in gpurun_out/p4prof${TAG}/.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$REPO/gpurun_out/p4prof${TAG:-}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for spec in ${SPECS:-C3-uk-2005:JAC:16 C4-sk-2005:JAC:16 C3-uk-2005:AA:16}; do
  IFS=: read cfg met hub <<< "$spec"
  name=${cfg%%-*}_${met}_${hub}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o tr -- \
    python3 $REPO/tools/sweep.py --config $cfg --metrics $met --hubs $hub --cpu-hubs "" --reps 2 \
    > $OUT/$name.jsonl 2> $OUT/$name.err
  rc=$?; echo "$name rc=$rc"; cat $OUT/$name.jsonl | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
  python3 $REPO/tools/kagg2.py $OUT/$name 2 > $OUT/$name.kagg.txt 2>&1; head -30 $OUT/$name.kagg.txt
done
exit 0
