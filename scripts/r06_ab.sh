#!/bin/bash
# Round-6 A/B of a runtime knob under the driver's command (config $2):
# alternating runs with ENV=A and ENV=B, one JSON line each.
#   bash scripts/r06_ab.sh TAG CONFIG VAR A B [REPS]
set -o pipefail
TAG=$1; C=$2; VAR=$3; A=$4; B=$5; REPS=${6:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq $REPS); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --config $C --no-cpu --e2e-steps 0 \
      > $OUT/ab_${VAR}_${v}_$r.json 2> $OUT/ab_${VAR}_${v}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/ab_${VAR}_${v}_$r.json').read().strip().splitlines()[-1]); print('$VAR=$v rep $r', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], d['host_ms_per_step'])"
  done
done
