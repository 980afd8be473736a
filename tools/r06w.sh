set -o pipefail
mkdir -p gpurun_out/r06w
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06w/prof -o create -- python3 -u $GRAFT_REPO_ROOT/tools/create_probe.py --repeat 1 > $GRAFT_REPO_ROOT/gpurun_out/r06w/probe.log 2>&1
