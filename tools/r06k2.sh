set -o pipefail
mkdir -p gpurun_out/r06k2
export NLP_TEST_REPORT_DIR=$GRAFT_REPO_ROOT/gpurun_out/r06k2
NLP_LONG_REFCHECK=1 timeout -k 10 800 python -u -m pytest -v --timeout 700 --timeout-method thread tests/test_gpu_c4.py -k "jaccard_h32 or adamic_adar_h32" --durations=5 > gpurun_out/r06k2/tests.log 2>&1
