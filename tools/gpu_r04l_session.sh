#!/bin/bash
# round-4 session l: survivor bitmask; SQ counters of the C4 JAC H=16 call's kernels
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04l STEPS=tests TESTS_LIMIT=600 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_c4.py" PYTEST_K="hash_path or c4_jaccard" tools/gpu_r04.sh || exit 1
TAG=r04l STEPS=sweep SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh || exit 1
TAG=r04l STEPS=sweeppmc PMC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" SWEEP_ARGS="--config C4-sk-2005 --metrics JAC --hubs 16 --cpu-hubs= --reps 1" tools/gpu_r04.sh
