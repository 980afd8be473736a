#!/bin/bash
# round-4 session z: kernel trace of C4 JAC / AA H=16
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04z STEPS=sweepprof SWEEP_ARGS="--config C4-sk-2005 --metrics JAC,AA --hubs 16 --cpu-hubs= --reps 2" tools/gpu_r04.sh
