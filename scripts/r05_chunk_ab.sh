#!/bin/bash
# Round-5 probe: chunk size under the driver's command (20 steps from an
# empty pipeline): one 10k chunk per batch (default) vs 5000 / 2500-problem
# chunks (DEPPY_CHUNK_PROBLEMS), config 2, interleaved, --no-cpu.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_chunk
mkdir -p $OUT
for rep in 1 2 3; do
  for v in 65536 5000 2500; do
    DEPPY_CHUNK_PROBLEMS=$v timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-steps 0 \
      > $OUT/c2_${v}_$rep.json 2> $OUT/c2_${v}_$rep.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/c2_${v}_$rep.json').read().strip().splitlines()[-1]); print('chunk $v rep $rep value', d['value'], 'ms', d['ms_per_step'], 'chunks', d['pipeline']['chunks_per_step'])"
  done
done
