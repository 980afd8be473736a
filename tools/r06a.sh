set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06a/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_dist.py tests/test_gpu_c1.py tests/test_gpu_parity.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r06a/tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06a/bench.json 2> gpurun_out/r06a/bench.err
