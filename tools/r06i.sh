set -o pipefail
mkdir -p gpurun_out/r06i
export NLP_TEST_REPORT_DIR=$PWD/gpurun_out/r06i
NLP_LONG_REFCHECK=1 timeout -k 10 1000 python -u -m pytest tests/test_gpu_c4.py -k "h32" -x -v --timeout 900 --timeout-method thread --durations=5 > gpurun_out/r06i/c4.log 2>&1
