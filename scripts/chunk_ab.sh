#!/bin/bash
# Config 2 under the driver's command (20 steps, warmup 5): chunk size
# (DEPPY_CHUNK_PROBLEMS: 10k = one chunk per step, the default; 5k, 2.5k)
# and jobs in flight (--depth), interleaved twice on one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-chunk_ab}
mkdir -p $OUT
for rep in 1 2; do
  for v in "-|0" "-|8" "-|24" "DEPPY_CHUNK_PROBLEMS=5000|0" "DEPPY_CHUNK_PROBLEMS=2500|0"; do
    e=${v%%|*}; d=${v##*|}; envs=""; [ "$e" != "-" ] && envs="$e"
    env $envs timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 5 --depth $d --kernel-steps 0 --no-cpu --e2e-steps 0 > $OUT/run.json 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/run.json').read().strip().splitlines()[-1]); print('[$e depth $d] config 2 h2h', d['value'], 'ms/step', d['ms_per_step'], d['config']['path'], d['pipeline']['chunks_per_step'])" | tee -a $OUT/ab.txt
  done
done
