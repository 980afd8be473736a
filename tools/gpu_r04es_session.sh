#!/bin/bash
# record-sort session: path-4 parity tests (incl. the 1M-vertex chain), C4 H=16 sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r04es STEPS=tests PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_dist.py" PYTEST_K="hash or short_list or h16_1m" TESTS_LIMIT=900 tools/gpu_r04.sh &&
TAG=r04es STEPS=sweep SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16,32 --cpu-hubs= --reps 2" tools/gpu_r04.sh &&
TAG=r04es STEPS=sweepprof SWEEP_ARGS="--config C4-sk-2005 --metrics JAC --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh
