set -o pipefail
mkdir -p gpurun_out/r06l
NLP_TRACE_HUB=1 timeout -k 10 240 python -u tools/sweep.py --config C4-sk-2005 --metrics AA --hubs 32 --cpu-hubs "" --reps 1 > gpurun_out/r06l/aa32_trace.log 2>&1
