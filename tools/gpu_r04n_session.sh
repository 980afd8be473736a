#!/bin/bash
# round-4 session n: pipelined bin-1 row queue (k_hp_rowb); parity and C4 H=16
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04n STEPS=tests TESTS_LIMIT=600 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_c4.py" PYTEST_K="hash_path or c4_jaccard_h16 or c4_adamic_adar_h16" tools/gpu_r04.sh || exit 1
TAG=r04n STEPS=sweepprof SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh
