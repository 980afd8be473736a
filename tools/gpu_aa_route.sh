#!/bin/bash
# Adamic-Adar / RA at large H: default routing (paths 1/2) vs forced path 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in 0 1; do
  if [ $f = 1 ]; then export NLP_HASH=1; fi
  timeout -k 10 400 python tools/sweep.py --metrics AA,RA --hubs ${HUBS:-16,64,256} --cpu-hubs "" --reps 2 \
    > gpurun_out/aa_route$f.jsonl 2> gpurun_out/aa_route$f.err || { echo "forced=$f failed"; exit 1; }
done
python - <<'PY'
import json
for f in (0, 1):
    for l in open("gpurun_out/aa_route%d.jsonl" % f):
        d = json.loads(l); print("forced", f, d["metric"], d["H"], d["path"], round(d["gpu_ms"], 2), d["predicted"])
PY
