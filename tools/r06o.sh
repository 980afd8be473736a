set -o pipefail
mkdir -p gpurun_out/r06o
( for i in $(seq 1 30); do sleep 45; date >> gpurun_out/r06o/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r06o/parity.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --sweep = --wp-steps 3 > gpurun_out/r06o/bench.log 2>&1
