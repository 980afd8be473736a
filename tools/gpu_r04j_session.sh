#!/bin/bash
# round-4 session j: first-order exclusion by the membership table for wide rows: path-4 parity,
# C4 JAC / AA H=16 with the factor swept, C3 JAC / AA H=16, kernel traces
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04j STEPS=tests TESTS_LIMIT=900 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_c4.py tests/test_gpu_c5.py" PYTEST_K="hash or star or c5 or c4" tools/gpu_r04.sh || exit 1
TAG=r04j STEPS=sweep SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2 --envs NLP_HASH_UX=8;NLP_HASH_UX=off;NLP_HASH_UX=2;NLP_HASH_UX=4;NLP_HASH_UX=16" tools/gpu_r04.sh || exit 1
TAG=r04j STEPS=sweepprof SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh || exit 1
mv gpurun_out/r04j/sweepprof gpurun_out/r04j/sweepprof_c4 && mv gpurun_out/r04j/sweepprof.log gpurun_out/r04j/sweepprof_c4.log
TAG=r04j STEPS=sweepprof SWEEP_ARGS="--config C3-uk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh
