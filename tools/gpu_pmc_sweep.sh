#!/bin/bash
# SQ counter passes over one tools/sweep.py call (kernel-level PMC), one rocprofv3
# run per pass.  PASSES="C1,C2,..;C3,.." SPEC=config:metric:H.  Output in gpurun_out/${TAG}/.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$REPO/gpurun_out/${TAG:-pmcsweep}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
IFS=: read cfg met hub <<< "$SPEC"
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
IFS=';' read -ra passes <<< "$PASSES"
for pc in "${passes[@]}"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc ${pc//,/ } --output-format csv -d $OUT/p$i -o pmc -- \
    python3 $REPO/tools/sweep.py --config $cfg --metrics $met --hubs $hub --cpu-hubs "" --reps 1 \
    > $OUT/p$i.jsonl 2> $OUT/p$i.err
  rc=$?; echo "pass $i ($pc) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/p$i.err; exit $rc; }
done
exit 0
