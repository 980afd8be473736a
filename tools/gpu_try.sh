set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "hash" > gpurun_out/pytest_hash.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/pytest_hash.log | head -30
if [ $rc -ne 0 ]; then exit $rc; fi
TRY_REPS=2 timeout -k 10 300 python -u tools/try_h.py JAC:16 AA:16 JAC:64 CN:1024 CN:0 > gpurun_out/try.log 2>&1
rc=$?; echo "try rc=$rc"; grep -v amdgpu.ids gpurun_out/try.log | cut -c1-300
exit $rc
