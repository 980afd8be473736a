set -o pipefail
mkdir -p gpurun_out/r06g2
( for i in $(seq 1 30); do sleep 45; date >> gpurun_out/r06g2/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --config C3-uk-2005 --metric AA --hub 16 --work-point none --sweep= --no-dropin > gpurun_out/r06g2/c3_aa16.log 2>&1 &&
timeout -k 10 400 python3 -u tools/sweep.py --config C4-sk-2005 --metrics JAC,CN --hubs 32,16,8 --cpu-hubs= --reps 2 > gpurun_out/r06g2/c4_sweep.log 2>&1
