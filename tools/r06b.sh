set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 120 ./tools/probe/alloc_probe > gpurun_out/r06b/alloc_probe.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "invalid_inputs or reference_api" -x -v --timeout 200 --timeout-method thread > gpurun_out/r06b/tests.log 2>&1
