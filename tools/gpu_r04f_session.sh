#!/bin/bash
# round-4 session f: path-4 parity (hash variants, star hub, C4, C5 range), then C4 H=16 and the C5 range timed
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04f STEPS=tests TESTS_LIMIT=900 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_c4.py tests/test_gpu_c5.py" PYTEST_K="hash or star or c4 or c5" tools/gpu_r04.sh || exit 1
TAG=r04f STEPS=sweep,c5prof SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh
