set -o pipefail
mkdir -p gpurun_out/r06m
( for i in $(seq 1 30); do sleep 45; date >> gpurun_out/r06m/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "hash or hub or adamic or resource" > gpurun_out/r06m/parity.log 2>&1 &&
NLP_TRACE_HUB=1 timeout -k 10 240 python -u tools/sweep.py --config C4-sk-2005 --metrics AA,RA --hubs 32,16 --cpu-hubs "" --reps 1 > gpurun_out/r06m/aa32_trace.log 2>&1 &&
timeout -k 10 240 python -u tools/sweep.py --config C4-sk-2005 --metrics AA,RA --hubs 32,16,8 --cpu-hubs "" --reps 2 > gpurun_out/r06m/aa_sweep.log 2>&1 &&
timeout -k 10 700 python -u -m pytest -x -v --timeout 650 --timeout-method thread tests/test_gpu_c4.py -k "adamic_adar_h32" > gpurun_out/r06m/c4aa32.log 2>&1
