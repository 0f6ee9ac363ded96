#!/bin/bash
# Config 2 (and 6) with one launch per residency class (DEPPY_CEILINGS=fine,
# merged only at equal residency) against the coarse default, the later
# launches of a chunk serial on its stream or spread over sibling lane
# streams (DEPPY_SPREAD=1).  Interleaved twice on one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-fine_ab}
mkdir -p $OUT
for rep in 1 2; do
  for cfg in 2 6; do
    for v in "-" "DEPPY_CEILINGS=fine DEPPY_BUCKET_MERGE=0.99" "DEPPY_CEILINGS=fine DEPPY_BUCKET_MERGE=0.99 DEPPY_SPREAD=1"; do
      envs=""; [ "$v" != "-" ] && envs="$v"
      env $envs timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 5 --kernel-steps 30 --no-cpu --e2e-steps 0 > $OUT/run.json 2>&1 || exit 1
      python3 -c "import json; d=json.loads(open('$OUT/run.json').read().strip().splitlines()[-1]); print('[$v] config $cfg', 'h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'serial_ms', d['kernel_only']['serial_launch_ms'], 'chunks', d['pipeline'])" | tee -a $OUT/ab.txt
    done
  done
done
