#!/bin/bash
# GPU tests and the driver's bench command, twice (8 lane streams on 8 hardware queues).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/kb5
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' $OUT/tests.log | head -20; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 3 > $OUT/bench_$i.json 2>&1 || { tail -5 $OUT/bench_$i.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_$i.json').read().strip().splitlines()[-1]); print('h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'e2e', d['end_to_end']['res_per_s'], 'latency', d['latency']['gpu_ms_median'], d['latency']['cpu_1thread_ms_median'], 'path', d['config']['path'], 'allocs', d['allocs_in_timed_region'])"
done
