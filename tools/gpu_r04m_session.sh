#!/bin/bash
# round-4 session m: record passes over 256-thread tiles; row-batch occupancy variants (after the table exclusion)
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04m STEPS=tests TESTS_LIMIT=600 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_c4.py" PYTEST_K="hash_path or c4_jaccard_h16" tools/gpu_r04.sh || exit 1
NLP_ES_NT=256 TAG=r04m2 STEPS=tests TESTS_LIMIT=600 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_c4.py" PYTEST_K="hash_path_vs_oracle and 0 or c4_jaccard_h16" tools/gpu_r04.sh || exit 1
TAG=r04m STEPS=sweep SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2 --envs NLP_ES_NT=512;NLP_ES_NT=256;NLP_HB_VAR=2;NLP_HB_VAR=3;NLP_HB_VAR=4;NLP_HB_VAR=1" tools/gpu_r04.sh
