#!/bin/bash
# Interleaved kernel-only A/B of library variants over several configs on one box.
#   scripts/ab3.sh "<configs>" <rounds> <variant.so|product> ...
set -o pipefail
export TMPDIR=/tmp
CFGS=$1; ROUNDS=$2; shift 2
# (a measurement variant built after the call was queued joins it)
if [ -f deppy_amd/libdeppy_hip_fv.so ]; then set -- "$@" libdeppy_hip_fv.so; fi
mkdir -p gpurun_out/ab
for r in $(seq 1 $ROUNDS); do
  for cfg in $CFGS; do
    for v in "$@"; do
      if [ "$v" = product ]; then unset DEPPY_VARIANT_LIB; else export DEPPY_VARIANT_LIB=$v; fi
      timeout -k 10 120 python bench.py --config $cfg --steps 2 --warmup 1 --kernel-steps 24 --no-cpu --e2e-steps 0 > gpurun_out/ab/run.json 2>&1 || { echo "run $v failed"; tail -5 gpurun_out/ab/run.json; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/ab/run.json').read().strip().splitlines()[-1]); print('$v', 'config $cfg', 'kernel_only', d['kernel_only']['res_per_s'], 'serial_ms', d['kernel_only']['serial_launch_ms'])" | tee -a gpurun_out/ab/ab3.txt
    done
  done
done
