#!/bin/bash
# The core pool's counter zeroed by the chunk's input copy (DEPPY_POOL_IN=1,
# default) against a 4-byte fill kernel on the stream before every chunk's
# launches (0): configs 2, 5 and 6 under the driver's command, interleaved
# twice on one box, after the GPU parity tests.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pool_ab}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for cfg in 2 5 6; do
    for v in 1 0; do
      DEPPY_POOL_IN=$v timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu --e2e-steps 0 > $OUT/run.json 2>&1 || exit 1
      python3 -c "import json; d=json.loads(open('$OUT/run.json').read().strip().splitlines()[-1]); print('[pool_in=$v] config $cfg h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'])" | tee -a $OUT/ab.txt
    done
  done
done
