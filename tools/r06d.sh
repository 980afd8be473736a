set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06d/smoke.log 2>&1 &&
timeout -k 10 400 python -u tools/create_probe.py --repeat 1 > gpurun_out/r06d/create.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c1.py tests/test_gpu_big_offsets.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r06d/tests.log 2>&1
