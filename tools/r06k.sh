set -o pipefail
mkdir -p gpurun_out/r06k
( for i in $(seq 1 30); do sleep 45; date >> gpurun_out/r06k/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 python -u tools/batch_all.py --out gpurun_out/r06k/batch_c2.json --ref-budget 200 --dropin-timeout 420 > gpurun_out/r06k/batch.log 2>&1
