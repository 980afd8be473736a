set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/sweep.py > gpurun_out/sweep_c2.jsonl 2> gpurun_out/sweep_c2.err
rc=$?; echo "rc=$rc"; python3 -c "
import json
for l in open('gpurun_out/sweep_c2.jsonl'):
    d=json.loads(l); print(d['metric'], d['H'], 'path', d['path'], 'gpu %.2f ms'%d['gpu_ms'], 'wedges %.3g'%d['wedges'], ('cpu %.0f ms x%.0f'%(d['cpu_ms'], d['speedup'])) if 'cpu_ms' in d else '')
"
exit $rc
