#!/bin/bash
# Iteration session: GPU parity suite (or PYTEST_K subset), the bench line,
# the rocprofv3 step timeline, then per-stage phase stamps (STAGES).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
mkdir -p gpurun_out/iter
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/iter/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/iter/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/iter/bench.json 2> gpurun_out/iter/bench.err \
  || { echo "bench failed"; tail -5 gpurun_out/iter/bench.err; exit 1; }
cut -c1-400 gpurun_out/iter/bench.json
bash tools/gpu_timeline.sh _iter > /dev/null && cat gpurun_out/tl_iter/step_timeline.txt || exit 1
if [ -n "${STAGES:-}" ]; then STAGES="$STAGES" bash tools/gpu_stamps.sh || exit 1; fi
