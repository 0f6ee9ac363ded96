#!/bin/bash
# A/B of the copy chain while an idle pipeline fills (DEPPY_COPY_CHAIN):
# host to host at the driver's 20 steps and at 100 (steady state).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/chain
mkdir -p $OUT
for rep in 1; do
for spec in "2 20" "3 20" "4 20" "5 20" "6 20"; do
  set -- $spec
  for ch in 0 64; do
    f=$OUT/c$1_s$2_ch${ch}_r$rep.json
    DEPPY_COPY_CHAIN_MB=$ch timeout -k 10 300 python bench.py --config $1 --steps $2 --warmup 5 --no-cpu --e2e-steps 0 --kernel-steps 3 > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('c$1 steps $2 chain $ch rep $rep h2h', d['value'])"
  done
done
done
