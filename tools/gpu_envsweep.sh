#!/bin/bash
# Kernel timeline (tools/gpu_timeline.sh) of the bench for each value of one
# knob: SWEEP_VAR=NLP_DX_BITS SWEEP_VALS="9 10 11" bash tools/gpu_envsweep.sh
# Optional PYTEST_K runs a subset of the GPU parity tests first.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"; mkdir -p gpurun_out
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "$PYTEST_K" > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
for v in $SWEEP_VALS; do
  echo "=== $SWEEP_VAR=$v"
  env "$SWEEP_VAR=$v" bash "$REPO/tools/gpu_timeline.sh" "_$v" | grep -E "rocprof rc|ms_per_step|k_sp|kernel time" | cut -c1-140 || exit 1
done
