#!/bin/bash
# Config 2 host to host: fill and drain at the driver's 20 steps vs longer runs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/c2steps
mkdir -p $OUT
for spec in "20 0" "100 0" "20 16" "100 16"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config 2 --steps $1 --warmup 5 --depth $2 --no-cpu --e2e-steps 0 --kernel-steps 20 > $OUT/c2_s$1_d$2.json 2>&1 || { tail -5 $OUT/c2_s$1_d$2.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c2_s$1_d$2.json').read().strip().splitlines()[-1]); print('steps $1 depth $2 h2h', d['value'], 'ko', d.get('kernel_only',{}).get('res_per_s'), d['config']['path'], d['pipeline'])"
done
