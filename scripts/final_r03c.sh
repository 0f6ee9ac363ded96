#!/bin/bash
# Round-3 closing check of the last build: the full GPU tests and smoke, the
# driver's bench command, and configs 4 and 5 (device-built lists, copy chain).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/final_c
mkdir -p $OUT
timeout -k 10 450 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2>&1 || { tail -5 $OUT/bench_c2.json; exit 1; }
for cfg in 4 5; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 20 --warmup 5 > $OUT/bench_c$cfg.json 2>&1 || { tail -5 $OUT/bench_c$cfg.json; exit 1; }
done
for f in $OUT/bench_c*.json; do
  python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['kernel_only']['res_per_s'] if d.get('kernel_only') else None, d['cpu_baseline']['value'] if d.get('cpu_baseline') else None, d.get('latency'), d['end_to_end']['res_per_s'] if d.get('end_to_end') else None, d.get('host_lowering_res_per_s'))"
done
