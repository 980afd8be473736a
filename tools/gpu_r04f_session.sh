#!/bin/bash
# round-4 session f: the path-4 call sequence of the hash tests under short limits first, then path-4
# parity (hash variants, star hub, C4, C5 range), then C4 H=16 and the C5 range timed
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04f; mkdir -p $OUT
for g in g3k edge; do
  NLP_HASH=1 NLP_HASH_EMIT=1 timeout -k 5 60 python3 -u tools/dbg_hang.py $g all > $OUT/dbg_$g.log 2>&1
  rc=$?; echo "dbg $g rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
TAG=r04f STEPS=tests TESTS_LIMIT=900 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_c4.py tests/test_gpu_c5.py" PYTEST_K="hash or star or c4 or c5" tools/gpu_r04.sh || exit 1
TAG=r04f STEPS=sweep,c5prof SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh
