#!/bin/bash
# Config 2 kernel-only rate against one-wavefront residency per CU: each
# launch's LDS request padded (DEPPY_LDS_PAD_KB) so fewer catalogs fit a CU.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r03_residency.jsonl
for pad in 0 20 23 27 32 40 54 80; do
  DEPPY_LDS_PAD_KB=$pad timeout -k 10 120 python bench.py --steps 2 --warmup 1 --kernel-steps 40 --no-cpu --e2e-steps 0 > gpurun_out/r03_res_$pad.json 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/r03_res_$pad.json').read().strip().split(chr(10))[-1]); print(json.dumps({'pad_kb':$pad,'per_cu':(160//$pad if $pad else 9),'kernel_res_per_s':d['kernel_only']['res_per_s'],'serial_launch_ms':d['kernel_only']['serial_launch_ms']}))" >> gpurun_out/r03_residency.jsonl
done
