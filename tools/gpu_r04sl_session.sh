#!/bin/bash
# short-list session: path-4 parity tests, C4 H=16 sweep with and without the class-ordered short lists, kernel profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r04sl STEPS=tests PYTEST_FILES=tests/test_gpu_parity.py PYTEST_K="hash or short_list" TESTS_LIMIT=900 tools/gpu_r04.sh &&
TAG=r04sl STEPS=sweep SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,CN,AA --hubs 16 --cpu-hubs= --reps 2 --envs NLP_DEBUG=1;NLP_HASH_SLIST=0" tools/gpu_r04.sh &&
TAG=r04sl STEPS=sweepprof SWEEP_ARGS="--config C4-sk-2005 --metrics JAC --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh
