#!/bin/bash
# Config 2/3 kernel-only and host-to-host rates by record form (P16D / U16 / int32).
set -o pipefail
mkdir -p gpurun_out
for cfg in 2 3; do for f in packed u16 i32; do
  timeout -k 10 150 python bench.py --config $cfg --record-form $f --steps 20 --warmup 5 --kernel-steps 40 --no-cpu --e2e-steps 0 > gpurun_out/r03_form_c${cfg}_$f.json 2>&1 || exit 1
done; done
