#!/bin/bash
# Multi-wave placements, current build against a variant library
# (DEPPY_VARIANT_LIB, scripts/mkvariant.sh): GPU parity tests of the current
# build, then interleaved on one box config-4 single-catalog latency (the
# same catalogs, scripts/c4_latency.py) and the config 4 / 5 bench lines.
#   usage: bash scripts/mw_ab.sh <tag> <variant lib> [catalogs]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-mw_ab}
VAR=${2:-libdeppy_hip_base.so}
M=${3:-20}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in new old; do
    envs=""; [ $v = old ] && envs="DEPPY_VARIANT_LIB=$VAR"
    env $envs timeout -k 10 300 python -u scripts/c4_latency.py $M > $OUT/c4lat_${v}_$rep.jsonl 2>&1 || exit 1
    echo "[$v] $(tail -1 $OUT/c4lat_${v}_$rep.jsonl)"
  done
done
for cfg in 4 5; do
  for v in new old; do
    envs=""; [ $v = old ] && envs="DEPPY_VARIANT_LIB=$VAR"
    env $envs timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --kernel-steps 12 --no-cpu --e2e-steps 0 > $OUT/c${cfg}_$v.json 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/c${cfg}_$v.json').read().strip().splitlines()[-1]); print('[$v] config $cfg', 'h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'serial_ms', d['kernel_only']['serial_launch_ms'])" | tee -a $OUT/ab.txt
  done
done
exit 0
