#!/bin/bash
# Kernel-only A/B of library variants on one box, interleaved:
#   scripts/ab.sh <config> <rounds> <variant.so|product> ...
# Each run: bench.py kernel-only rate (records resident, 8 batches in flight).
set -o pipefail
export TMPDIR=/tmp
CFG=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out/ab
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    if [ "$v" = product ]; then unset DEPPY_VARIANT_LIB; else export DEPPY_VARIANT_LIB=$v; fi
    timeout -k 10 120 python bench.py --config $CFG --steps 3 --warmup 1 --kernel-steps 40 --no-cpu --e2e-steps 0 > gpurun_out/ab/run.json 2>&1 || { echo "run $v failed"; cat gpurun_out/ab/run.json | tail -5; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab/run.json').read().strip().splitlines()[-1]); print('$v', 'config $CFG', 'kernel_only', d['kernel_only']['res_per_s'], 'serial_ms', d['kernel_only']['serial_launch_ms'], 'h2h', d['value'])" | tee -a gpurun_out/ab/ab_c$CFG.txt
  done
done
