#!/bin/bash
# round-4 session r: drop-in header fix (count query) checked (test + bench), C3 JAC / AA H=16
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04r STEPS=tests TESTS_LIMIT=400 PYTEST_FILES="tests/test_gpu_dropin.py tests/test_gpu_multi.py" tools/gpu_r04.sh || exit 1
TAG=r04r STEPS=sweep SWEEP_ARGS="--config C3-uk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh || exit 1
TAG=r04r STEPS=bench BENCH_LIMIT=900 tools/gpu_r04.sh
