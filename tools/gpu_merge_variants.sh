#!/bin/bash
# 8-rank rehearsal (tools/shard_emul.py) with variant builds of libnlp.so:
#   LIBS="libnlp.so libnlp_mw1024.so" bash tools/gpu_merge_variants.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for l in ${LIBS:-libnlp.so}; do
  NLP_LIB_PATH=$PWD/neighborhood-link-prediction-openmp_amd/$l timeout -k 10 400 python tools/shard_emul.py --ranks ${RANKS:-8} --steps 5 \
    > gpurun_out/merge_$l.log 2>&1 || { echo "$l failed"; tail -3 gpurun_out/merge_$l.log; exit 1; }
  echo "== $l: $(tail -1 gpurun_out/merge_$l.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("merge_ms", round(d["merge_ms"],4), "equal", d["equal_single_range"], "predict_ms", [round(x,3) for x in d["predict_ms_per_rank"]][:3])')"
done
