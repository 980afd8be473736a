#!/bin/bash
# Path-4 check: hash-path parity tests, then the large-H sweep with and
# without the bin-0 table-size tiers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "hash or large_hub" -p no:cacheprovider > gpurun_out/pytest_hash.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_hash.log
[ $rc -ne 0 ] && exit $rc
for t in 1 0; do
  NLP_HASH_TIERS=$t timeout -k 10 300 python tools/sweep.py --metrics ${METRICS:-JAC,CN} --hubs ${HUBS:-16,64,0} --cpu-hubs "" --reps 2 \
    > gpurun_out/sweep_tiers$t.jsonl 2> gpurun_out/sweep_tiers$t.err || { echo "sweep tiers=$t failed"; exit 1; }
done
python - <<'PY'
import json
for t in (1, 0):
    for l in open("gpurun_out/sweep_tiers%d.jsonl" % t):
        d = json.loads(l); print("tiers", t, d["metric"], d["H"], d["path"], round(d["gpu_ms"], 2), d["predicted"])
PY
