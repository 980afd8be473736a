#!/bin/bash
# round-4 session g: the hub pass's segment histograms (k_hh_hist / k_hh_group):
# path-4 parity (hash variants, star hub, C5 range), then the C5 range (CN, AA) traced
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04g STEPS=tests TESTS_LIMIT=900 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_c5.py tests/test_gpu_multi.py" PYTEST_K="hash or star or c5 or c4_jac or partitions" tools/gpu_r04.sh || exit 1
TAG=r04g STEPS=c5prof tools/gpu_r04.sh || exit 1
mv gpurun_out/r04g/c5prof gpurun_out/r04g/c5prof_cn && mv gpurun_out/r04g/c5prof.log gpurun_out/r04g/c5prof_cn.log
TAG=r04g STEPS=c5prof RANGE_ARGS="--metric AA" tools/gpu_r04.sh
