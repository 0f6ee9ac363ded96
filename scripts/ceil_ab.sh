#!/bin/bash
# Config 2/3/5 kernel-only and host-to-host rates: LDS bucket ceilings A/B
# (12-per-CU bucket on/off, bucket merge ratio).
set -o pipefail
mkdir -p gpurun_out/ceil
for v in "DEPPY_NO_CEIL12=1" "DEPPY_BUCKET_MERGE=0.5" "DEPPY_BUCKET_MERGE=0.85" "DEPPY_BUCKET_MERGE=0"; do
  for c in 2 5; do
    env $v timeout -k 10 200 python -u bench.py --config $c --steps 30 --kernel-steps 8 --no-cpu > gpurun_out/ceil/$c.$v.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ceil/$c.$v.json')); print('$c', '$v', d['value'], d['kernel_only']['res_per_s'], d['kernel_only']['serial_launch_ms'])"
  done
done
