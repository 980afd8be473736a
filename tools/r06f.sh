set -o pipefail
mkdir -p gpurun_out/r06f
NLP_BUILD_TRACE=1 timeout -k 10 400 python -u tools/create_probe.py --repeat 3 > gpurun_out/r06f/create.log 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06f/bench.json 2> gpurun_out/r06f/bench.err
