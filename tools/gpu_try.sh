set -u
mkdir -p gpurun_out
NLP_HOSTPROF=1 TRY_REPS=3 timeout -k 10 300 python -u tools/try_h.py JAC:8 JAC:16:NLP_HASH=0 > gpurun_out/try.log 2>&1
rc=$?; echo "try rc=$rc"; grep -v amdgpu.ids gpurun_out/try.log | cut -c1-200
exit $rc
