set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c1.py > gpurun_out/r06e/tests.log 2>&1 &&
timeout -k 10 300 python3 -u tools/create_probe.py --repeat 2 > gpurun_out/r06e/probe.log 2>&1
