set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "evaluation or driver or edge_cases or reference_api" > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/pytest_new.log | head -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log | cut -c1-900
exit $rc
