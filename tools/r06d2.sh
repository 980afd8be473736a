set -o pipefail
mkdir -p gpurun_out/r06d2
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r06d2/tests.log 2>&1 &&
timeout -k 10 300 python3 -u tools/create_probe.py --repeat 1 > gpurun_out/r06d2/probe.log 2>&1
