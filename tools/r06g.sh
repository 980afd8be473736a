set -o pipefail
mkdir -p gpurun_out/r06g
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread --durations=40 > gpurun_out/r06g/tests.log 2>&1
