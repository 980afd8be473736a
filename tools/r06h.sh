set -o pipefail
mkdir -p gpurun_out/r06h
timeout -k 10 480 python -u tools/ref_time.py --calls JAC:32,AA:32 --timeout 200 > gpurun_out/r06h/ref_time.log 2>&1 &&
timeout -k 10 680 python -u tools/batch_all.py --out gpurun_out/r06h/batch_c2.json --ref-budget 180 --dropin-timeout 300 > gpurun_out/r06h/batch.log 2>&1
