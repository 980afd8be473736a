set -o pipefail
mkdir -p gpurun_out/r06s
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "hash or short or golden or multigraph" > gpurun_out/r06s/tests.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --sweep = --wp-steps 2 > gpurun_out/r06s/bench.log 2>&1
