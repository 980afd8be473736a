#!/bin/bash
# each step a fresh process under its own short limit; continues past timeouts of the single call (no GPU fault)
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/dbg3; mkdir -p $OUT
export NLP_HASH=1 NLP_HASH_EMIT=1 NLP_HASH_STATS=1
for spec in "NLP_HASH_ONE=0 NLP_HASH_WIN=0" "NLP_HASH_WIN=0" "NLP_HASH_ONE=0" "X=1"; do
  echo "== $spec" >> $OUT/log
  env $spec timeout -k 5 20 python3 -u tools/dbg_hang.py edge 0 2 40 >> $OUT/log 2>&1
  rc=$?; echo "rc=$rc" >> $OUT/log
  [ $rc -eq 0 ] || [ $rc -eq 124 ] || exit $rc
done
