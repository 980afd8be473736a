#!/bin/bash
# round-4 session y: 128-thread rows for the 2048-entry bin-1 tier (counts and AA / RA); parity and C4 / C3 H=16
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04y STEPS=tests TESTS_LIMIT=600 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_c4.py" PYTEST_K="hash_path or c4_jaccard_h16 or c4_adamic_adar_h16" tools/gpu_r04.sh || exit 1
TAG=r04y STEPS=sweep SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 3" tools/gpu_r04.sh || exit 1
mv gpurun_out/r04y/sweep.log gpurun_out/r04y/sweep_c4.log
TAG=r04y STEPS=sweep SWEEP_ARGS="--config C3-uk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh
