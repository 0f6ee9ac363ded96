#!/bin/bash
# Round-4 baseline on one box: GPU parity tests, smoke, the driver's bench
# command (config 2) and the kernel-only rates of configs 2/3/6.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04_base}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2>$OUT/bench_c2.err || exit 1
tail -c 600 $OUT/bench_c2.json
for cfg in 3 6; do
  timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --kernel-steps 30 --no-cpu --e2e-steps 0 > $OUT/c$cfg.json 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('$OUT/c$cfg.json').read().strip().splitlines()[-1]); print('config $cfg', 'h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'serial_ms', d['kernel_only']['serial_launch_ms'])"
done
exit 0
