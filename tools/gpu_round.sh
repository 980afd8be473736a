#!/bin/bash
# Round-end GPU session: full GPU parity suite, the default bench line, the
# rocprofv3 kernel timeline/stats of the bench, and the PMC traffic passes.
# Everything lands in gpurun_out/round/ (copy what is judged into profiles/).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT=gpurun_out/round
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
bash tools/gpu_timeline.sh _round > /dev/null && cp gpurun_out/tl_round/step_timeline.txt $OUT/ && \
  cp "$(find gpurun_out/tl_round -name '*kernel_stats.csv' | head -1)" $OUT/bench_kernel_stats.csv || exit 1
cat $OUT/step_timeline.txt
bash tools/gpu_pmc.sh _round || exit 1
python tools/pmc_summary.py gpurun_out/pmc_round r02 > $OUT/pmc_summary.json && head -c 600 $OUT/pmc_summary.json
