#!/bin/bash
# round-4 session w: smoke, then the kernel trace and the FETCH_SIZE / WRITE_SIZE passes of the bench command
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04w; mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
TAG=r04w STEPS=prof,pmc tools/gpu_r04.sh
