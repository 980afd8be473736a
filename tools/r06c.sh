set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 200 ./tools/probe/alloc_probe > gpurun_out/r06c/alloc_probe.log 2>&1 &&
NLP_BUILD_TRACE=1 timeout -k 10 400 python -u tools/create_probe.py --repeat 2 > gpurun_out/r06c/create.log 2>&1
