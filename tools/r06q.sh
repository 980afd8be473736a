set -o pipefail
mkdir -p gpurun_out/r06q
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c1.py tests/test_gpu_multi.py > gpurun_out/r06q/tests.log 2>&1 &&
NLP_BUILD_TRACE=1 timeout -k 10 300 python3 -u tools/create_probe.py --repeat 2 > gpurun_out/r06q/probe.log 2>&1 &&
TAG=r06q STEPS=bench BENCH_LIMIT=600 bash tools/gpu_session.sh
