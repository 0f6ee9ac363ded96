#!/bin/bash
# Device-built watch lists for OLM-scale records (watch_build.hip): the GPU
# tests that touch multi-wave records, then config 4 and 5 with the lists
# built on the device (default) and on the host (DEPPY_HOST_WATCHES=1).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/dl
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread \
  -k "olm or wide or watch_boundary or config4 or queued" > $OUT/tests_sel.log 2>&1
rc=$?; tail -1 $OUT/tests_sel.log; [ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' $OUT/tests_sel.log | head -20; exit 1; }
for c in 4 5; do
  for hw in 0 1; do
    DEPPY_HOST_WATCHES=$hw timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --cpu-seconds 2 > $OUT/bench_c${c}_hw$hw.json 2>&1 || { tail -5 $OUT/bench_c${c}_hw$hw.json; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/bench_c${c}_hw$hw.json').read().strip().splitlines()[-1]); print('c$c hw$hw h2h', d['value'], 'ko', d.get('kernel_only',{}).get('res_per_s'), 'forms', d['config'].get('record_forms'), 'pcie', d.get('pcie'), 'e2e', d['end_to_end']['res_per_s'], 'low', d.get('host_lowering_res_per_s'))"
  done
done
