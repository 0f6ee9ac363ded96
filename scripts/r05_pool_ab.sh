#!/bin/bash
# Round-5 A/B: the core pool's counter zeroed by the chunk's H2D copy (default)
# vs a fill kernel ahead of each chunk's launches (DEPPY_POOL_MEMSET=1), the
# driver's command on configs 2, 6 and 5, interleaved, --no-cpu, no
# end-to-end leg.  GPU parity tests first.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_pool
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -1 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit 1
for cfg in 2 6 5; do
  for rep in 1 2 3; do
    for v in 0 1; do
      DEPPY_POOL_MEMSET=$v timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --config $cfg --no-cpu --e2e-steps 0 \
        > $OUT/c${cfg}_${v}_$rep.json 2> $OUT/c${cfg}_${v}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$OUT/c${cfg}_${v}_$rep.json').read().strip().splitlines()[-1]); print('config $cfg pool_memset $v rep $rep value', d['value'], 'ms', d['ms_per_step'], 'kernel_only', d['kernel_only']['res_per_s'], 'exact', d.get('verified_bit_exact_vs_oracle'))"
    done
  done
done
