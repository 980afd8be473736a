#!/bin/bash
# round-4 session s: C3 JAC H=16 by exclusion factor; kernel trace of the default
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04s STEPS=sweep SWEEP_ARGS="--config C3-uk-2005 --metrics JAC --hubs 16 --cpu-hubs= --reps 2 --envs NLP_HASH_UX=1;NLP_HASH_UX=off;NLP_HASH_UX=0;NLP_HASH_UX=4;NLP_HASH_STATS=1" tools/gpu_r04.sh || exit 1
TAG=r04s STEPS=sweepprof SWEEP_ARGS="--config C3-uk-2005 --metrics JAC --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh
