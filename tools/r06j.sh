set -o pipefail
mkdir -p gpurun_out/r06j
export NLP_TEST_REPORT_DIR=$PWD/gpurun_out/r06j
( for i in $(seq 1 30); do sleep 45; date >> gpurun_out/r06j/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
NLP_LONG_REFCHECK=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_c4.py -k "h32" -x -v --timeout 600 --timeout-method thread --durations=5 > gpurun_out/r06j/c4.log 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06j/sweepprof -o sweep -- python3 $GRAFT_REPO_ROOT/tools/sweep.py --config C4-sk-2005 --metrics AA,JAC --hubs 16,32 --cpu-hubs "" --reps 2 > $GRAFT_REPO_ROOT/gpurun_out/r06j/sweep.log 2>&1)
