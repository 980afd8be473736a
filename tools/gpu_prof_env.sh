#!/bin/bash
# Kernel traces of tools/sweep.py calls under several environment settings:
# RUNS="name|ENV=.. ENV2=..|config:metric:H ..." entries separated by ';'.
# Output in gpurun_out/${TAG}/<name>/.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$REPO/gpurun_out/${TAG:-envprof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra runs <<< "$RUNS"
for run in "${runs[@]}"; do
  IFS='|' read name envs specs <<< "$run"
  for spec in $specs; do
    IFS=: read cfg met hub <<< "$spec"
    tag=${name}_${cfg%%-*}_${met}_${hub}
    env $envs true || exit 9
    export $envs
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o tr -- \
      python3 $REPO/tools/sweep.py --config $cfg --metrics $met --hubs $hub --cpu-hubs "" --reps 2 \
      > $OUT/$tag.jsonl 2> $OUT/$tag.err
    rc=$?
    for kv in $envs; do unset ${kv%%=*}; done
    echo "$tag rc=$rc"; cut -c1-260 $OUT/$tag.jsonl
    [ $rc -ne 0 ] && exit $rc
    python3 $REPO/tools/kagg2.py $OUT/$tag 2 > $OUT/$tag.kagg.txt 2>&1; head -14 $OUT/$tag.kagg.txt
  done
done
exit 0
