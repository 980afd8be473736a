set -o pipefail
mkdir -p gpurun_out/r06k
( for i in $(seq 1 30); do sleep 45; date >> gpurun_out/r06k/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
NLP_TRACE_HUB=1 timeout -k 10 240 python -u tools/sweep.py --config C4-sk-2005 --metrics AA --hubs 32 --cpu-hubs "" --reps 1 > gpurun_out/r06k/aa32_trace.log 2>&1 &&
timeout -k 10 900 python -u tools/batch_all.py --out gpurun_out/r06k/batch_c2.json --ref-budget 200 --dropin-timeout 420 > gpurun_out/r06k/batch.log 2>&1
