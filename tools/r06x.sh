set -o pipefail
mkdir -p gpurun_out/r06x
timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "two_level or folded_into_order or hash_path_vs_oracle and (22 or 23 or 24)" > gpurun_out/r06x/tests.log 2>&1 &&
NLP_TRACE_RUNS=1 timeout -k 10 400 python3 -u tools/sweep.py --config C4-sk-2005 --metrics JAC,CN,AA --hubs 16 --cpu-hubs '' --reps 3 --envs 'NLP_ES_RUNS=0;NLP_ES_RUNS=1' > gpurun_out/r06x/sweep.log 2>&1
