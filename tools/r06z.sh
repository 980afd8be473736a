set -o pipefail
mkdir -p gpurun_out/r06z
timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "two_level or folded_into_order or hash_path_vs_oracle and (22 or 23 or 24)" > gpurun_out/r06z/tests.log 2>&1 &&
NLP_TRACE_RUNS=1 timeout -k 10 500 python3 -u tools/sweep.py --config C4-sk-2005 --metrics JAC,CN,AA --hubs 16 --cpu-hubs '' --reps 5 --envs 'NLP_ES_RUNS=1;NLP_ES_RUNS=2;NLP_ES_RUNS=1,NLP_ES8_NT=512;NLP_ES_RUNS=2,NLP_ES8_NT=512' > gpurun_out/r06z/sweep.log 2>&1
