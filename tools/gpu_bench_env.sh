#!/bin/bash
# Bench ms/step under several environment settings (one bench process each):
#   BENCH_ENVS="X=1 NLP_END_EVENT=1" bash tools/gpu_bench_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for e in ${BENCH_ENVS:-X=1}; do
  r=$(env ${e//,/ } NLP_HOSTPROF=100 timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-300} --warmup 20 --no-cpu-baseline 2>&1) || { echo "$e failed"; echo "$r" | tail -5; exit 1; }
  echo "== $e: $(echo "$r" | grep -o '"ms_per_step": [0-9.]*') | $(echo "$r" | grep 'host us' | tail -1)"
done
