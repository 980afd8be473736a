#!/bin/bash
# Round-end measurement: the default bench line (with the CPU baseline), its
# kernel trace (stats + step timeline), and the FETCH_SIZE / WRITE_SIZE passes
# of the same command.  Output in gpurun_out/${TAG}.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG=${TAG:-r03_final}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/bench.err; exit $rc; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print({k: d[k] for k in ('ms_per_step','value','predicted','score_ms','select_ms','host_overhead_ms')})
print(d['roofline']); print(d['cpu_baseline']); print([(x['H'], round(x['ms'],3), x['path']) for x in d['hub_sweep']])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
  python3 $REPO/bench.py --steps 20 --warmup 3 --no-cpu-baseline --sweep = > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 $REPO/tools/prof_summary.py $OUT/prof/bench_kernel_trace.csv > $OUT/step_timeline.txt; cat $OUT/step_timeline.txt
mkdir -p $OUT/pmc
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc/p$i" -o pmc -- \
    python3 "$REPO/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --sweep = > "$OUT/pmc/p$i.log" 2>&1 \
    || { echo "pmc pass $i failed"; exit 1; }
  echo "pmc pass $i ok ($grp)"
done
exit 0
