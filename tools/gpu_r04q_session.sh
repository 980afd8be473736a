#!/bin/bash
# round-4 session q: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the bench command, and C3 AA H=16 line
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04q STEPS=prof,pmc tools/gpu_r04.sh || exit 1
TAG=r04q_c3 STEPS=bench BENCH_LIMIT=500 BENCH_ARGS="--config C3-uk-2005 --metric AA --hub 16 --work-point none --sweep = --no-dropin" tools/gpu_r04.sh
