#!/bin/bash
# GPU tests; kernel-only A/B product vs the no-BCP-counter build (configs 2, 3);
# the latency line of a full bench run.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/kb4
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' $OUT/tests.log | head -20; exit 1; }
bash scripts/ab3.sh "2 3" 2 product libdeppy_hip_novis.so || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 2 > $OUT/bench.json 2>&1 || { tail -5 $OUT/bench.json; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('h2h', d['value'], 'latency', d['latency'], 'e2e', d['end_to_end']['res_per_s'], d['end_to_end']['cpu_res_per_s'])"
