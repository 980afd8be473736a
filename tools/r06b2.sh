set -o pipefail
mkdir -p gpurun_out/r06b2
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r06b2/tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_c4.py -k "jaccard_h16" > gpurun_out/r06b2/c4.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06b2/prof -o create -- python3 -u $GRAFT_REPO_ROOT/tools/create_probe.py --repeat 1 > $GRAFT_REPO_ROOT/gpurun_out/r06b2/probe.log 2>&1
