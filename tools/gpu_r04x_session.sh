#!/bin/bash
# round-4 session x: the default bench line of the final build
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04x STEPS=bench BENCH_LIMIT=1100 tools/gpu_r04.sh
