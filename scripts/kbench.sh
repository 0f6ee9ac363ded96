#!/bin/bash
# One measurement pass of the current build: GPU parity tests, then the
# kernel-only rate (records resident in HBM) of configs 2, 3 and 6, and the
# SQ instruction mix of config 2 (one PMC pass).  Output: gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-kb}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
for cfg in 2 3 6; do
  timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --kernel-steps 30 --no-cpu --e2e-steps 0 > $OUT/c$cfg.json 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('$OUT/c$cfg.json').read().strip().splitlines()[-1]); print('config $cfg', 'h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'serial_ms', d['kernel_only']['serial_launch_ms'])"
done
bash scripts/pmc_sq_r02.sh 2 > $OUT/sq.log 2>&1 || exit 1
python3 scripts/sq_summary.py gpurun_out/sq > $OUT/sq.json && cat $OUT/sq.json | head -30
exit 0
