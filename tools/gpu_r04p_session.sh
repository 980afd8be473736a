#!/bin/bash
# round-4 session p: the default bench line (headline, work point, CPU baselines, drop-in)
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04p STEPS=bench BENCH_LIMIT=1100 tools/gpu_r04.sh
