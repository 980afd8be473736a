set -o pipefail
mkdir -p gpurun_out/r06u
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r06u/tests.log 2>&1 &&
timeout -k 10 400 python3 -u tools/create_probe.py --envs "NLP_TRANSPOSE_LSD8=1;NLP_TRANSPOSE_LSD8=0;NLP_TRANSPOSE_LSD8=1" > gpurun_out/r06u/probe.log 2>&1
