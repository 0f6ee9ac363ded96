#!/bin/bash
# Round-5 A/B: copy chaining while the pipeline fills (DEPPY_COPY_CHAIN_MB:
# default 64 MB threshold vs 1 = every chunk), the driver's command on
# configs 2 and 6, interleaved, --no-cpu, no end-to-end leg.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_chain
mkdir -p $OUT
for cfg in 2 6; do
  for rep in 1 2 3; do
    for v in 64 1; do
      DEPPY_COPY_CHAIN_MB=$v timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --config $cfg --no-cpu --e2e-steps 0 \
        > $OUT/c${cfg}_${v}_$rep.json 2> $OUT/c${cfg}_${v}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$OUT/c${cfg}_${v}_$rep.json').read().strip().splitlines()[-1]); print('config $cfg chain_mb $v rep $rep value', d['value'], 'ms', d['ms_per_step'])"
    done
  done
done
