#!/bin/bash
# round-4 session h: hub-pass direct counters: path-4 parity, item statistics, C5 range CN / AA traced
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04h; mkdir -p $OUT
TAG=r04h STEPS=tests TESTS_LIMIT=900 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_c4.py tests/test_gpu_c5.py" PYTEST_K="hash or star or c5 or c4" tools/gpu_r04.sh || exit 1
NLP_HH_STATS=1 timeout -k 10 200 python3 tools/range_call.py --reps 0 > $OUT/stats_cn.log 2>&1 || exit 1
NLP_HH_STATS=1 timeout -k 10 200 python3 tools/range_call.py --reps 0 --metric AA > $OUT/stats_aa.log 2>&1 || exit 1
TAG=r04h STEPS=c5prof tools/gpu_r04.sh || exit 1
mv $OUT/c5prof $OUT/c5prof_cn && mv $OUT/c5prof.log $OUT/c5prof_cn.log
TAG=r04h STEPS=c5prof RANGE_ARGS="--metric AA" tools/gpu_r04.sh
TAG=r04h STEPS=sweep SWEEP_ARGS="--config C4-sk-2005 --metrics JAC --hubs 16 --cpu-hubs= --reps 2 --envs NLP_HB_XP=0;NLP_HB_XP=1;NLP_HB_XP=2;NLP_HB_XP=4;NLP_HB_XP=12;NLP_HB_XP=15;NLP_HASH_HUB_MIN=1;NLP_HASH_ROWB=0;NLP_ES_VAR=1" tools/gpu_r04.sh
TAG=r04h STEPS=sweepprof SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh
