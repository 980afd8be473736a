#!/bin/bash
# round-4 session v: record passes stage (u, w) as one word; parity and C4 / C3 H=16
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04v STEPS=tests TESTS_LIMIT=600 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_c4.py" PYTEST_K="hash_path_vs_oracle or c4_jaccard_h16 or c4_adamic_adar_h16 or order" tools/gpu_r04.sh || exit 1
TAG=r04v STEPS=sweep SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 3" tools/gpu_r04.sh
