#!/bin/bash
# Config 4 host to host: the pipeline's fill and drain at 20 steps vs longer
# runs, and jobs in flight.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/c4steps
mkdir -p $OUT
for spec in "20 0" "80 0" "80 8" "80 24"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config 4 --steps $1 --warmup 5 --depth $2 --no-cpu --e2e-steps 0 --kernel-steps 5 > $OUT/c4_s$1_d$2.json 2>&1 || { tail -5 $OUT/c4_s$1_d$2.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c4_s$1_d$2.json').read().strip().splitlines()[-1]); print('steps $1 depth $2 h2h', d['value'], 'ko', d.get('kernel_only',{}).get('res_per_s'), d['config']['path'], 'pcie', d.get('pcie',{}).get('h2d_GBs'))"
done
