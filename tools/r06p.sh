set -o pipefail
mkdir -p gpurun_out/r06p
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "symmetry or multigraph or golden" > gpurun_out/r06p/tests.log 2>&1 &&
NLP_BUILD_TRACE=1 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --sweep = --wp-steps 2 > gpurun_out/r06p/bench.log 2>&1
