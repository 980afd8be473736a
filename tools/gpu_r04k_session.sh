#!/bin/bash
# round-4 session k: survivor lists by k_dc_* (default) vs the one-pass build; the exclusion factor
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04k STEPS=tests TESTS_LIMIT=900 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_c4.py tests/test_gpu_c5.py" PYTEST_K="hash or star or c5 or c4" tools/gpu_r04.sh || exit 1
TAG=r04k STEPS=sweep SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2 --envs NLP_HASH_UX=2;NLP_HASH_UX=1;NLP_HASH_UX=0;NLP_HASH_ONE=1,NLP_HASH_UX=1" tools/gpu_r04.sh || exit 1
TAG=r04k STEPS=sweepprof SWEEP_ARGS="--config C4-sk-2005 --metrics JAC --hubs 16 --cpu-hubs= --reps 2 --envs NLP_HASH_UX=1" tools/gpu_r04.sh
