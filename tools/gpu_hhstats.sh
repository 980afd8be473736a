cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/hhs
NLP_HH_STATS=1 timeout -k 10 200 python3 tools/range_call.py --reps 0 > gpurun_out/hhs/cn.log 2>&1 && NLP_HH_STATS=1 timeout -k 10 200 python3 tools/range_call.py --reps 0 --metric AA > gpurun_out/hhs/aa.log 2>&1
