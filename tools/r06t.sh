set -o pipefail
mkdir -p gpurun_out/r06t
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "two_level or folded_into_order or hash_path_vs_oracle or all_candidates" > gpurun_out/r06t/tests.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06t/prof -o sweep -- python3 -u $GRAFT_REPO_ROOT/tools/sweep.py --config C4-sk-2005 --metrics JAC,CN,AA --hubs 16,32 --cpu-hubs '' --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r06t/sweep.log 2>&1
