#!/bin/bash
# Round 5: NotSatisfiable by deletion with recursive model rotation (oracle
# and kernel together).  GPU tests, config 5 / 2 driver-command bench lines,
# then the config-4 counters of the 2-byte watch entries (r05_c4_pmc.sh).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_rot
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
for cfg in 5 2; do
  timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 5 --cpu-seconds 5 > $OUT/bench_c$cfg.json 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/bench_c$cfg.json').read().strip().splitlines()[-1]); print('config $cfg', d['value'], d['kernel_only']['res_per_s'], d['kernel_only']['serial_launch_ms'], d['latency']['gpu_ms_median'], d['latency']['gpu_ms_p90'], d['cpu_baseline']['value'], d['verified_bit_exact_vs_oracle'])"
done
bash scripts/r05_c4_pmc.sh
